"""Folds rocprofv3 --pmc CSVs (gpurun_out/pmc_*/**/*counter_collection.csv) into one JSON:
mean counter value per dispatch, per kernel.  FETCH_SIZE / WRITE_SIZE are in KB as reported."""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
acc = collections.defaultdict(lambda: collections.defaultdict(list))
prefix = sys.argv[4] if len(sys.argv) > 4 else "pmc"  # (run directories <root>/<prefix>_<pass>)
for path in glob.glob(os.path.join(root, prefix + "_*", "**", "*counter_collection.csv"), recursive=True):
    per = collections.defaultdict(float)  # (kernel, dispatch, counter) -> summed value
    with open(path) as f:
        for row in csv.DictReader(f):
            k = row["Kernel_Name"].split("(")[0]
            per[(k, row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
    for (k, _, c), v in per.items():
        acc[k][c].append(v)
out = {k: {c: sum(v) / len(v) for c, v in sorted(cs.items())} for k, cs in sorted(acc.items())}
batch = int(sys.argv[2]) if len(sys.argv) > 2 else None
lanes = int(sys.argv[3]) if len(sys.argv) > 3 else 1
head = os.environ.get("SDSJ_HEAD", "")
json.dump({"note": "rocprofv3 --pmc, mean per dispatch (bench.py --steps 2 --warmup 1); one dispatch = one lane "
                   "of the batch (batch / lanes images)", "batch": batch, "lanes": lanes, "head": head,
           "kernels": out}, sys.stdout, indent=1)
