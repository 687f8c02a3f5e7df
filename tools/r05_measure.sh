#!/bin/bash
# Round-5 measurement at HEAD, in three calls (each step under its own limit; a timeout / signal stops
# the rest of the call):
#   tools/r05_measure.sh a        bench lines of configs[1] / [2] / [4], progressive, chroma samplings,
#                                 the decode service, the collate-side batched consumer (f1) at 8 / 16 workers
#   tools/r05_measure.sh b        the reference's loader shape: service / Pillow / null at 2, 4, 8, 16
#                                 workers, and random_resize through the service at 8 and 16
#   tools/r05_measure.sh c HEAD   rocprof kernel stats (4 lanes, 1 lane) + PMC at configs[1] and mixed512
#                                 (HEAD = the last kernel-source commit, recorded in the PMC summaries),
#                                 and an 8-rank rehearsal on one GPU
part=${1:-a}
tag=r05
if [ "$part" = a ]; then
  tools/gpu_steps.sh \
    "bench|300|python bench.py > gpurun_out/${tag}_bench.json" \
    "mixed|200|python bench.py --workload mixed512 --no-cpu-baseline > gpurun_out/${tag}_bench_mixed512.json" \
    "e2e|300|python bench.py --workload e2e512 --no-cpu-baseline > gpurun_out/${tag}_bench_e2e512.json" \
    "prog|300|python tools/prog_bench.py 4096 > gpurun_out/${tag}_prog_bench.json" \
    "sampling|300|python tools/sampling_bench.py 4096 > gpurun_out/${tag}_sampling.jsonl" \
    "svc|200|python tools/service_bench.py 3 1 2 4 8 16 32" \
    "f1w8|120|python tools/batched_bench.py 2048 5 256 8" \
    "f1w16|120|python tools/batched_bench.py 2048 5 256 16"
elif [ "$part" = b ]; then
  for w in 2 4 8 16; do
    for kind in service pil null; do
      tools/gpu_steps.sh "ps_${kind}_w$w|120|python -u tools/persample_bench.py 512 4 ${kind}_fork_workers${w}_pinned" || exit $?
    done
  done
  for w in 8 16; do
    tools/gpu_steps.sh "ps_servicerr_w$w|120|python -u tools/persample_bench.py 512 4 servicerr_fork_workers${w}_pinned" || exit $?
  done
else
  export SDSJ_HEAD=${2:-}
  tools/gpu_steps.sh \
    "prof|900|tools/profile_round.sh $tag" \
    "pmcmixed|600|BATCH=8192 PMC_OUT=pmc_mixed512.json tools/pmc.sh --workload mixed512" \
    "ranks8|300|python bench.py --gpus 8 --backend gloo --batch 2048 --steps 3 --warmup 1 --no-cpu-baseline --roofline-steps 1 > gpurun_out/${tag}_rehearsal_8ranks_1gpu.json"
fi
