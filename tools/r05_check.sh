#!/bin/bash
# Round-5 check run: GPU suite, configs[1] x2, configs[2], configs[4] with the restated downloader, the
# ADVICE r04 six-slot case against the round-4 library (expected to fail there), and the per-sample
# loader-shape modes with the service client's phase profile.
rm -f gpurun_out/svc_profile.jsonl
tools/gpu_steps.sh \
  "gputest|600|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "bench|180|python bench.py --no-cpu-baseline" \
  "bench2|180|python bench.py --no-cpu-baseline" \
  "mixed|180|python bench.py --no-cpu-baseline --workload mixed512" \
  "e2e|300|python bench.py --no-cpu-baseline --workload e2e512" \
  "r04six|180|SDSJ_LIBRARY=sds_amd/lib/exp/libsdsj_r04.so python -u -m pytest tests/test_gpu_parity.py -q -k six_table --timeout 120 --timeout-method thread" \
  "persample|400|SDS_AMD_SERVICE_PROFILE=gpurun_out/svc_profile.jsonl python -u tools/persample_bench.py 512 4 service,pil,null" || exit $?
tools/ab.sh 3 "" base=sds_amd/lib/exp/libsdsj_base.so head=product && \
SDSJ_HEAD=${SDSJ_HEAD:-wip} tools/pmc.sh
