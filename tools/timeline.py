"""Concurrency profile of a 4-lane bench run from a rocprofv3 kernel trace (<dir>/**/*kernel_trace.csv):
over the timed steps (bench.py: 1 gate + W warm-up steps, then K timed steps, each with 4 k_parse
dispatches -- one per lane), the time during which 0 / 1 / 2 / 3 / 4+ sdsj kernels ran at once, and for
the time with exactly one kernel running, which kernel it was (the pipeline's serial part).
    python tools/timeline.py <trace dir> [warmup] [steps] [lanes]"""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    warm = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    lanes = int(sys.argv[4]) if len(sys.argv) > 4 else 4
    path = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    ks = []
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"]
        if "sdsj" not in n:
            continue
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n.split("(")[0].replace("void ", "").replace("sdsj::", "")))
    ks.sort()
    parses = [s for s, _, n in ks if n.startswith("k_parse")]
    t0 = parses[(1 + warm) * lanes]
    t1 = parses[(1 + warm + steps) * lanes]
    ev = []
    for s, e, n in ks:
        s, e = max(s, t0), min(e, t1)
        if e > s:
            ev.append((s, 1, n))
            ev.append((e, -1, n))
    ev.sort()
    run = collections.Counter()
    by_conc = collections.Counter()
    alone = collections.Counter()
    busy = collections.Counter()
    last = t0
    for t, k, n in ev:
        dt = t - last
        c = sum(run.values())
        by_conc[min(c, 4)] += dt
        if c == 1:
            alone[next(iter(+run))] += dt
        for m in +run:
            busy[m] += dt * run[m]
        run[n] += k
        last = t
    tot = t1 - t0
    print(f"window {tot / 1e6:.1f} ms ({steps} steps: {tot / 1e6 / steps:.2f} ms per step)")
    for c in sorted(by_conc):
        print(f"  {c}{'+' if c == 4 else ''} kernels running: {by_conc[c] / tot * 100:5.1f} %")
    print("time with one kernel running, by kernel (ms):")
    for n, v in alone.most_common(12):
        print(f"  {n:45s} {v / 1e6:7.2f}")
    print("kernel busy time in the window (ms, summed over concurrent dispatches):")
    for n, v in busy.most_common(14):
        print(f"  {n:45s} {v / 1e6:7.2f}")


if __name__ == "__main__":
    main()
