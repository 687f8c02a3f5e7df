#!/bin/bash
# Single-lane kernel-trace stats of one bench workload (GPU box); prints the per-kernel averages.
# usage: tools/prof_quick.sh <tag> [bench args]
set -e
export TMPDIR=/tmp
tag=$1
shift
rm -rf gpurun_out/pq_$tag
SDSJ_LANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pq_$tag -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/pq_$tag.log 2>&1 || echo "bench exited with $? (stats still read)"
python3 - gpurun_out/pq_$tag/run_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows if "sdsj" in r["Name"]) / 1e3 / max(int(r["Calls"]) for r in rows if "sdsj" in r["Name"])
print(f"sdsj kernels per call: {tot:.1f} us")
for r in rows:
    if "sdsj" in r["Name"] and float(r["AverageNs"]) > 20000:
        print(f"  {r['Name'].split('(')[0][:40]:40s} {float(r['AverageNs']) / 1e3:9.1f} us")
PY
