#!/bin/bash
# r05: decode-once cost probe A/B, then the service engine count at 2 / 4 / 8 / 16 workers.
export TMPDIR=/tmp
tools/ab.sh 3 "" head=product doprobe=sds_amd/lib/exp/libsdsj_doprobe.so || exit $?
for e in 2 3 4; do
  for w in 2 4 8 16; do
    SDS_AMD_SERVICE_ENGINES=$e timeout -k 10 120 python -u tools/persample_bench.py 512 4 service_fork_workers${w}_pinned > gpurun_out/svc_e${e}_w${w}.log 2>&1 || exit $?
    echo "engines $e $(grep -h '^{' gpurun_out/svc_e${e}_w${w}.log)" >> gpurun_out/svc_sweep.log
  done
done
