#!/bin/bash
# A/B product vs sds_amd/lib/exp/libsdsj_base.so on configs[1] and configs[2], then the GPU suite.
export TMPDIR=/tmp
tools/ab.sh ${ROUNDS:-3} "" base=sds_amd/lib/exp/libsdsj_base.so head=product || exit $?
mv gpurun_out/ab.log gpurun_out/ab_vga.log
tools/ab.sh 2 "--workload mixed512" base=sds_amd/lib/exp/libsdsj_base.so head=product || exit $?
mv gpurun_out/ab.log gpurun_out/ab_mixed.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1; echo "gputest rc=$?" >> gpurun_out/ab_vga.log
