"""Kernel statistics from a rocprofv3 SQLite output (rocpd tables): per kernel name, calls, total and
mean duration (ns), optionally the per-call timeline of one engine call (the gaps between kernels).
    python tools/rocpd_stats.py results.db [--timeline N]"""
import collections
import sqlite3
import sys


def main():
    db = sys.argv[1]
    c = sqlite3.connect(db)
    names = {r[0]: r[1] for r in c.execute("select id, display_name from rocpd_info_kernel_symbol")}
    rows = list(c.execute("select kernel_id, start, end from rocpd_kernel_dispatch order by start"))
    agg = collections.defaultdict(lambda: [0, 0])
    for k, s, e in rows:
        agg[names[k]][0] += 1
        agg[names[k]][1] += e - s
    tot = sum(v[1] for v in agg.values())
    print(f"{'kernel':70s} {'calls':>7s} {'total_ms':>10s} {'mean_us':>9s} {'pct':>6s}")
    for n, (cnt, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{n[:70]:70s} {cnt:7d} {t / 1e6:10.3f} {t / cnt / 1e3:9.2f} {100 * t / tot:6.1f}")
    if "--timeline" in sys.argv:
        n = int(sys.argv[sys.argv.index("--timeline") + 1])
        first = [i for i, (k, s, e) in enumerate(rows) if "k_parse" in names[k]]
        if len(first) > n + 1:
            a, b = first[n], first[n + 1]
            t0 = rows[a][1]
            for k, s, e in rows[a:b]:
                print(f"  +{(s - t0) / 1e3:8.1f} us  {(e - s) / 1e3:7.1f} us  {names[k][:70]}")


if __name__ == "__main__":
    main()
