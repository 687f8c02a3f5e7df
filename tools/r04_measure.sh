#!/bin/bash
# Round-4 measurement at HEAD, in two calls (each under gpurun's per-call limit; each step under its own
# limit, a timeout / signal stops the rest):
#   tools/r04_measure.sh a        bench lines of configs[1] / [2] / [4], the decode service, per-sample loader
#   tools/r04_measure.sh b HEAD   rocprof kernel stats (4 lanes, 1 lane) + PMC at vga256 and mixed512
#                                 (HEAD = the last kernel-source commit, recorded in the PMC summaries),
#                                 and an 8-rank rehearsal on one GPU
part=${1:-a}
tag=r04
if [ "$part" = a ]; then
  tools/gpu_steps.sh \
    "bench|300|python bench.py > gpurun_out/${tag}_bench.json" \
    "mixed|200|python bench.py --workload mixed512 --no-cpu-baseline > gpurun_out/${tag}_bench_mixed512.json" \
    "e2e|200|python bench.py --workload e2e512 --no-cpu-baseline > gpurun_out/${tag}_bench_e2e512.json" \
    "svc|200|python tools/service_bench.py 3 1 2 4 8 16 32" \
    "persample|300|for m in service_fork_workers2_pinned service_fork_workers8_pinned service_fork_workers16_pinned main_process_per_sample; do python tools/persample_bench.py 512 4 \$m || exit 1; done"
else
  export SDSJ_HEAD=${2:-}
  tools/gpu_steps.sh \
    "prof|700|tools/profile_round.sh $tag" \
    "pmcmixed|300|BATCH=2048 PMC_OUT=pmc_mixed512.json tools/pmc.sh --workload mixed512" \
    "ranks8|300|python bench.py --gpus 8 --backend gloo --batch 2048 --steps 3 --warmup 1 --no-cpu-baseline --roofline-steps 1 > gpurun_out/${tag}_rehearsal_8ranks_1gpu.json"
fi
