#!/bin/bash
# A/B of library variants on the progressive path: tools/prog_bench.py (no CPU baseline) per variant,
# alternating, `rounds` times; one JSON line per run into gpurun_out/prog_ab.log.
# usage: tools/prog_ab.sh rounds batch name=lib ...   (lib "product" = the in-tree build)
set -e
export TMPDIR=/tmp
rounds=$1; shift
batch=$1; shift
mkdir -p gpurun_out
for r in $(seq 1 $rounds); do
  for spec in "$@"; do
    name=${spec%%=*}; lib=${spec#*=}
    if [ "$lib" = "product" ]; then unset SDSJ_LIBRARY; else export SDSJ_LIBRARY=$lib; fi
    echo -n "$name " >> gpurun_out/prog_ab.log
    timeout -k 10 120 python3 tools/prog_bench.py $batch nocpu 2> gpurun_out/prog_ab_$name.err | tail -1 >> gpurun_out/prog_ab.log
    tail -1 gpurun_out/prog_ab.log
  done
done
unset SDSJ_LIBRARY
