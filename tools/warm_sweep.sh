#!/bin/bash
# Entropy warm-up sweep at the bench's default batch (SDSJ_WARM_BITS overrides the plan's warm-up for
# every image): one bench line per setting into gpurun_out/warm.log.  usage: tools/warm_sweep.sh bits... [-- bench args]
mkdir -p gpurun_out
args=()
vals=()
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then shift; args=("$@"); break; fi
  vals+=("$1"); shift
done
for r in 1 2; do
  for w in "${vals[@]}"; do
    if [ "$w" = "default" ]; then unset SDSJ_WARM_BITS; else export SDSJ_WARM_BITS=$w; fi
    timeout -k 10 150 python3 bench.py --no-cpu-baseline "${args[@]}" > gpurun_out/warm.json 2>/dev/null
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/warm.json') if l.startswith('{')][-1]); s=d['stage_ms_per_step_single_lane']; print('warm $w', d['value'], 'spec', s['entspec'], 'sync', s['entsync'])" | tee -a gpurun_out/warm.log
  done
done
