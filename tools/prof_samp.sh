#!/bin/bash
# Single-lane kernel-trace stats of tools/sampling_bench.py for one chroma sampling (GPU box).
# usage: tools/prof_samp.sh <4:2:2|4:4:4|gray|4:2:0>
set -e
export TMPDIR=/tmp
tag=$(echo "$1" | tr -d ':')
rm -rf gpurun_out/ps_$tag
SDSJ_LANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ps_$tag -o run -- \
  python3 tools/sampling_bench.py 4096 "$1" > gpurun_out/ps_$tag.log 2>&1
python3 - gpurun_out/ps_$tag/run_kernel_stats.csv "$1" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print(sys.argv[2])
for r in rows:
    if "sdsj" in r["Name"] and float(r["AverageNs"]) > 20000:
        print(f"  {r['Name'].split('(')[0][:40]:40s} {float(r['AverageNs']) / 1e3:9.1f} us  calls {r['Calls']}")
PY
