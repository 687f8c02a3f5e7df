#!/bin/bash
# configs[1] at the bench's batch (65,536) with 1 / 2 / 3 / 4 engine lanes (SDSJ_LANES), alternating, 2 rounds
# usage: tools/r05_lanes65k.sh [lanes ...]
export TMPDIR=/tmp
for r in 1 2; do
  for n in ${@:-1 2 3 4}; do
    SDSJ_LANES=$n timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/l_$n.json 2> gpurun_out/l_$n.err || exit $?
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/l_$n.json') if l.startswith('{')][-1]); print('lanes $n', d['value'], d['ms_per_step'])" >> gpurun_out/lanes65k.log
  done
done
