#!/bin/bash
# configs[2] (mixed512) at the batches given (default 2,048 / 4,096), alternating, 2 rounds
export TMPDIR=/tmp
for r in 1 2; do
  for b in ${@:-2048 4096}; do
    timeout -k 10 240 python3 bench.py --no-cpu-baseline --workload mixed512 --batch $b > gpurun_out/m_$b.json 2> gpurun_out/m_$b.err || exit $?
    python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/m_$b.json') if l.startswith('{')][-1]); print('mixed batch $b', d['value'], d['ms_per_step'])" >> gpurun_out/batch.log
  done
done
