#!/bin/bash
# Engine lanes per batch (SDSJ_LANES) at the bench's default batch: one line per setting into
# gpurun_out/lanes.log.  usage: tools/lanes_sweep.sh lanes... [-- bench args]
mkdir -p gpurun_out
args=()
vals=()
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then shift; args=("$@"); break; fi
  vals+=("$1"); shift
done
for r in 1 2; do
  for l in "${vals[@]}"; do
    SDSJ_LANES=$l timeout -k 10 150 python3 bench.py --no-cpu-baseline "${args[@]}" > gpurun_out/lanes.json 2>/dev/null
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/lanes.json') if l.startswith('{')][-1]); print('lanes $l', d['value'], d['ms_per_step'])" | tee -a gpurun_out/lanes.log
  done
done
