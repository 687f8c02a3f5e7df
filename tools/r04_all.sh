#!/bin/bash
# Round-4 GPU session in one call (each step under its own limit; a timeout / signal stops the rest):
# the GPU suite, the decode service (raw and in DataLoader workers), kernel A/B, the driver-style bench
# lines of configs[1] / [2] / [4], rocprof kernel stats + PMC at HEAD, and an 8-rank rehearsal on one GPU.
# usage: tools/r04_all.sh <tag> [variant specs for tools/ab.sh ...]
tag=${1:-r04}; shift
ab_specs="$*"
steps=(
  "gputest|600|python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread"
  "svc|200|python tools/service_bench.py 4 1 2 4 8 16"
  "persample|300|python tools/persample_bench.py 512 5 service_fork_workers8_pinned && python tools/persample_bench.py 512 5 service_fork_workers16_pinned && python tools/persample_bench.py 512 5 service_fork_workers2_pinned && python tools/persample_bench.py 512 5 main_process_per_sample"
  "bench|200|python bench.py > gpurun_out/${tag}_bench.json"
  "mixed|200|python bench.py --workload mixed512 --no-cpu-baseline > gpurun_out/${tag}_bench_mixed512.json"
  "e2e|200|python bench.py --workload e2e512 --no-cpu-baseline > gpurun_out/${tag}_bench_e2e512.json"
)
if [ -n "$ab_specs" ]; then steps+=("ab|500|tools/ab.sh 2 \"\" base=product $ab_specs"); fi
steps+=("prof|700|tools/profile_round.sh $tag")
steps+=("ranks8|300|python bench.py --gpus 8 --backend gloo --batch 2048 --steps 3 --warmup 1 --no-cpu-baseline --roofline-steps 1 > gpurun_out/${tag}_rehearsal_8ranks_1gpu.json")
tools/gpu_steps.sh "${steps[@]}"
exit $?
