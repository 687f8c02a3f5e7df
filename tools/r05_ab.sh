#!/bin/bash
# A/B of the product library against sds_amd/lib/exp/libsdsj_base.so (+ extra name=lib pairs), then the
# GPU suite on the product.
export TMPDIR=/tmp
tools/ab.sh ${ROUNDS:-3} "" base=sds_amd/lib/exp/libsdsj_base.so head=product "$@" || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1; echo "gputest rc=$?" >> gpurun_out/ab.log
