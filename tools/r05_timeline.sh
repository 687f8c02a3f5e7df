#!/bin/bash
# 4-lane kernel trace of configs[1] (batch as given), then the concurrency profile of the last 10 steps.
export TMPDIR=/tmp
B=${1:-32768}
rm -rf gpurun_out/tl
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --roofline-steps 1 --batch $B > gpurun_out/tl.log 2>&1 || exit $?
python3 -c "import json; d=json.loads([l for l in open('gpurun_out/tl.log') if l.startswith('{')][-1]); print('bench ms_per_step', d['ms_per_step'], 'value', d['value'])" > gpurun_out/timeline.txt
python3 tools/timeline.py gpurun_out/tl 3 10 4 >> gpurun_out/timeline.txt
