#!/bin/bash
# GPU suite on the product, then an A/B of variants on configs[1] and configs[2].
# usage: tools/r05_ab4.sh name=lib ...   (ROUNDS, MROUNDS: rounds per workload)
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1
rc=$?; echo "gputest rc=$rc" > gpurun_out/ab_vga.log
[ $rc -ne 0 ] && exit $rc
tools/ab.sh ${ROUNDS:-2} "" "$@" || exit $?
cat gpurun_out/ab.log >> gpurun_out/ab_vga.log
rm -f gpurun_out/ab.log
tools/ab.sh ${MROUNDS:-1} "--workload mixed512" "$@" || exit $?
mv gpurun_out/ab.log gpurun_out/ab_mixed.log
