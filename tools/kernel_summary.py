"""Summarise a rocprofv3 kernel-trace database: per-kernel total / count / mean, optionally only
kernels dispatched between two markers of a repeated pattern. Usage:
  python tools/kernel_summary.py gpurun_out/x/y_results.db [--top 25] [--grep NAME]"""
import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--grep", default=None)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    agg = defaultdict(lambda: [0.0, 0])
    for name, dur in c.execute("select name, duration from kernels"):
        if a.grep and a.grep not in name:
            continue
        k = name.split("(")[0][:90]
        agg[k][0] += dur / 1e3
        agg[k][1] += 1
    tot = sum(v[0] for v in agg.values())
    print(f"{'total_us':>12} {'pct':>6} {'count':>7} {'mean_us':>9}  kernel")
    for k, (t, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:a.top]:
        print(f"{t:12.1f} {100 * t / tot:6.2f} {n:7d} {t / n:9.2f}  {k}")
    print(f"{tot:12.1f} total")


if __name__ == "__main__":
    main()
