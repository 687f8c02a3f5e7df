#!/bin/bash
for v in product s1024w2000 s768w3000 s1024w4000 s512w2500; do
  if [ $v = product ]; then unset SDSJ_LIBRARY; else export SDSJ_LIBRARY=sds_amd/lib/exp/libsdsj_$v.so; fi
  echo -n "$v "; timeout -k 10 60 python tools/latency_probe.py 300 2>/dev/null | grep engine
done
