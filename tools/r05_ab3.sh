#!/bin/bash
# GPU suite first (new code paths), then A/B product vs base on configs[1] and configs[2].
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1
rc=$?; echo "gputest rc=$rc" > gpurun_out/ab_vga.log
[ $rc -ge 124 ] && exit $rc
tools/ab.sh ${ROUNDS:-3} "" base=sds_amd/lib/exp/libsdsj_base.so head=product || exit $?
cat gpurun_out/ab.log >> gpurun_out/ab_vga.log
tools/ab.sh 2 "--workload mixed512" base=sds_amd/lib/exp/libsdsj_base.so head=product || exit $?
mv gpurun_out/ab.log gpurun_out/ab_mixed.log
