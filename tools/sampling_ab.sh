#!/bin/bash
# A/B of library variants on one chroma sampling (tools/sampling_bench.py), alternating, `rounds`
# times.  usage: tools/sampling_ab.sh rounds sampling name=lib ...   (lib "product" = the in-tree build)
set -e
export TMPDIR=/tmp
rounds=$1; shift
samp=$1; shift
for r in $(seq 1 $rounds); do
  for spec in "$@"; do
    name=${spec%%=*}; lib=${spec#*=}
    if [ "$lib" = "product" ]; then unset SDSJ_LIBRARY; else export SDSJ_LIBRARY=$lib; fi
    echo "$name $(timeout -k 10 120 python3 tools/sampling_bench.py 4096 $samp | tail -1)"
  done
done
