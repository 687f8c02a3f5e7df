#!/bin/bash
# Per-sample latency (tools/latency_probe.py) of the product and of experiment libraries
# sds_amd/lib/exp/libsdsj_<name>.so; one line per library into gpurun_out/mhlat.log.
# usage: tools/mh_latency.sh name ...
set -o pipefail
mkdir -p gpurun_out
for v in product "$@"; do
  if [ "$v" = product ]; then unset SDSJ_LIBRARY; else export SDSJ_LIBRARY=sds_amd/lib/exp/libsdsj_$v.so; fi
  echo "$v $(timeout -k 10 60 python tools/latency_probe.py 300 | tail -1)" >> gpurun_out/mhlat.log || exit 1
done
