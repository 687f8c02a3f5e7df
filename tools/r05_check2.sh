#!/bin/bash
# r05 second check: GPU suite, A/B against the round-4 library, PMC, and the service at 16 workers with
# 2 / 4 / 8 engines (batch sizes traced).
tools/gpu_steps.sh \
  "gputest|600|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "mixed|180|python bench.py --no-cpu-baseline --workload mixed512" \
  "svc16_e8|200|SDSJ_SERVICE_TRACE=1 SDS_AMD_SERVICE_ENGINES=8 python -u tools/persample_bench.py 512 4 service_fork_workers16" \
  "svc16_e4|200|SDSJ_SERVICE_TRACE=1 SDS_AMD_SERVICE_ENGINES=4 python -u tools/persample_bench.py 512 4 service_fork_workers16" \
  "svc16_e2|200|SDSJ_SERVICE_TRACE=1 SDS_AMD_SERVICE_ENGINES=2 python -u tools/persample_bench.py 512 4 service_fork_workers16" || exit $?
tools/ab.sh 3 "" r04=sds_amd/lib/exp/libsdsj_r04.so head=product && \
SDSJ_HEAD=${SDSJ_HEAD:-wip} tools/pmc.sh
