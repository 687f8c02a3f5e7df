#!/bin/bash
# A/B of library variants on the GPU box: bench.py (no CPU baseline) per variant, alternating,
# `rounds` times; one line per run "name value stage_ms..." into gpurun_out/ab.log.
# usage: tools/ab.sh rounds "bench args" name=lib ...   (lib "product" = the in-tree build)
set -e
export TMPDIR=/tmp
rounds=$1; shift
args=$1; shift
mkdir -p gpurun_out
for r in $(seq 1 $rounds); do
  for spec in "$@"; do
    name=${spec%%=*}; lib=${spec#*=}
    if [ "$lib" = "product" ]; then unset SDSJ_LIBRARY; else export SDSJ_LIBRARY=$lib; fi
    timeout -k 10 120 python3 bench.py --no-cpu-baseline $args > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err
    python3 - "$name" gpurun_out/ab_$name.json >> gpurun_out/ab.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
st = d.get("stage_ms_per_step_single_lane", {})
print(sys.argv[1], d["value"], " ".join(f"{k}={v}" for k, v in st.items() if v > 0.05))
PY
    tail -1 gpurun_out/ab.log
  done
done
unset SDSJ_LIBRARY
