#!/bin/bash
# Round measurements on the GPU box (replaces the per-round rNN_*.sh scripts).  Every GPU step runs under
# its own time limit through tools/gpu_steps.sh; a step ending in a signal / timeout stops the call.
#
#   tools/measure.sh suite                   GPU test suite + smoke()
#   tools/measure.sh lines TAG               bench lines: configs[1] (CPU baseline), configs[2] and configs[4]
#                                            (each with its CPU baseline), progressive, chroma samplings,
#                                            the decode service, the f1 batched consumer at 8 / 16 workers
#   tools/measure.sh loader TAG              the reference's loader shape: service / Pillow / null at 2-16
#                                            workers (tools/persample_bench.py)
#   tools/measure.sh profile TAG HEAD        rocprof kernel stats (4 lanes, 1 lane) + PMC at configs[1] and
#                                            configs[2] (HEAD = the kernel-source commit, recorded in the PMC
#                                            summaries) + an 8-rank gloo rehearsal on one GPU
#   tools/measure.sh ab ROUNDS "ARGS" name=lib ...   A/B of library builds (tools/ab.sh; lib "product" = in-tree)
#   tools/measure.sh sweep batch|mbatch|lanes VALUE ...   configs[1] batch, configs[2] batch, or engine lanes
# Outputs land under gpurun_out/ (TAG_*.json / *.log); copy what is to be kept into profiles/.
export TMPDIR=/tmp
mkdir -p gpurun_out
part=${1:-suite}
shift || true
case "$part" in
  suite)
    tools/gpu_steps.sh \
      "gputest|600|python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread" \
      "smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'"
    ;;
  lines)
    tag=${1:-rNN}
    tools/gpu_steps.sh \
      "bench|300|python bench.py > gpurun_out/${tag}_bench.json" \
      "mixed|300|python bench.py --workload mixed512 > gpurun_out/${tag}_bench_mixed512.json" \
      "e2e|300|python bench.py --workload e2e512 > gpurun_out/${tag}_bench_e2e512.json" \
      "prog|300|python tools/prog_bench.py 4096 > gpurun_out/${tag}_prog_bench.json" \
      "sampling|300|python tools/sampling_bench.py 4096 > gpurun_out/${tag}_sampling.jsonl" \
      "svc|200|python tools/service_bench.py 3 1 2 4 8 16 32" \
      "f1w8|120|python tools/batched_bench.py 2048 5 256 8" \
      "f1w16|120|python tools/batched_bench.py 2048 5 256 16"
    ;;
  loader)
    for w in 2 4 8 16; do
      for kind in service pil null; do
        tools/gpu_steps.sh "ps_${kind}_w$w|120|python -u tools/persample_bench.py 512 4 ${kind}_fork_workers${w}_pinned" || exit $?
      done
    done
    ;;
  profile)
    tag=${1:-rNN}
    export SDSJ_HEAD=${2:-}
    tools/gpu_steps.sh \
      "prof|900|tools/profile_round.sh $tag" \
      "pmcmixed|600|BATCH=8192 PMC_OUT=pmc_mixed512.json tools/pmc.sh --workload mixed512" \
      "ranks8|300|python bench.py --gpus 8 --backend gloo --batch 2048 --steps 3 --warmup 1 --no-cpu-baseline --roofline-steps 1 > gpurun_out/${tag}_rehearsal_8ranks_1gpu.json"
    ;;
  ab)
    tools/ab.sh "$@"
    ;;
  sweep)
    kind=$1
    shift
    for r in 1 2; do
      for v in "$@"; do
        case "$kind" in
          batch) env=""; args="--batch $v" ;;
          mbatch) env=""; args="--workload mixed512 --batch $v" ;;
          lanes) env="SDSJ_LANES=$v"; args="" ;;
          *) echo "unknown sweep $kind"; exit 2 ;;
        esac
        env $env timeout -k 10 240 python3 bench.py --no-cpu-baseline $args > gpurun_out/sw_${kind}_$v.json 2> gpurun_out/sw_${kind}_$v.err || exit $?
        python3 -c "import json; d=json.loads([l for l in open('gpurun_out/sw_${kind}_$v.json') if l.startswith('{')][-1]); print('$kind $v', d['value'], d['ms_per_step'])" >> gpurun_out/sweep.log
      done
    done
    ;;
  *)
    echo "usage: tools/measure.sh suite|lines|loader|profile|ab|sweep ..."
    exit 2
    ;;
esac
