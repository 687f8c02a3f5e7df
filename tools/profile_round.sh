#!/bin/bash
# Round profile artifacts (run on the GPU box): rocprofv3 kernel-trace stats of the bench command at the
# default 4 lanes and at 1 lane (the roofline's unit), then PMC counters (separate passes, no tracing).
# Every dispatch is a full batch (--no-pixel-check: the pixel check's extra batches stay out of the averages).
# Outputs under gpurun_out/prof_<tag>*/ and gpurun_out/pmc.json.  usage: tools/profile_round.sh <tag> [bench args]
set -e
export TMPDIR=/tmp
tag=${1:-rNN}
shift || true
rm -rf gpurun_out/prof_$tag gpurun_out/prof_${tag}_l1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pixel-check $* > gpurun_out/prof_$tag.log 2>&1
SDSJ_LANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_l1 -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pixel-check $* > gpurun_out/prof_${tag}_l1.log 2>&1
timeout -k 10 900 tools/pmc.sh $* > gpurun_out/pmc_run.log 2>&1
