#!/bin/bash
# Unstuff-kernel A/B (round 4): one-lane kernel stats (tools/prof_quick.sh) of the product and of
# experiment libraries sds_amd/lib/exp/libsdsj_<name>.so on vga256 and mixed512; the k_us_* lines
# go to gpurun_out/us_ab.log.
# usage: tools/us_ab.sh name ...
set -e
mkdir -p gpurun_out
for w in ${US_WORKLOADS:-vga256 mixed512}; do
  for v in product "$@"; do
    if [ "$v" = product ]; then unset SDSJ_LIBRARY; else export SDSJ_LIBRARY=sds_amd/lib/exp/libsdsj_$v.so; fi
    tools/prof_quick.sh us_${v}_$w --workload $w > gpurun_out/us_${v}_$w.txt
    echo "$w $v $(grep -E "kernels per call|${US_PAT:-k_us_}" gpurun_out/us_${v}_$w.txt | tr -s ' ' | tr '\n' ' ')" >> gpurun_out/us_ab.log
  done
done
