#!/bin/bash
# configs[1] at the batches given (default 16,384 / 24,576 / 32,768; rows 100,000), alternating, 2 rounds
# usage: tools/r05_batch.sh [batch ...]
export TMPDIR=/tmp
for r in 1 2; do
  for b in ${@:-16384 24576 32768}; do
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --batch $b > gpurun_out/b_$b.json 2> gpurun_out/b_$b.err || exit $?
    python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/b_$b.json') if l.startswith('{')][-1]); print('batch $b', d['value'], d['ms_per_step'])" >> gpurun_out/batch.log
  done
done
