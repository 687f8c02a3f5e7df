#!/bin/bash
# Per-call latency (tools/latency_probe.py) of library variants on the GPU box.
# usage: tools/lat_ab.sh name ...   (name "product" = the in-tree build, else sds_amd/lib/exp/libsdsj_<name>.so)
for v in "$@"; do
  if [ "$v" = product ]; then unset SDSJ_LIBRARY; else export SDSJ_LIBRARY=sds_amd/lib/exp/libsdsj_$v.so; fi
  echo -n "$v "; timeout -k 10 60 python tools/latency_probe.py 300 2>/dev/null | grep engine
done
