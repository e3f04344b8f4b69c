"""Per-kernel breakdown of ONE optimizer step from a rocprofv3 kernel trace (the last complete step:
between the last two AdamW launches), so init / warm-up kernels do not distort the picture.
  python tools/step_profile.py gpurun_out/prof/bench_kernel_trace.csv [--top 30]"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--marker", default="adam_mt")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    # an optimizer step may launch the marker several times back to back (one per param group):
    # cluster adjacent launches; the step is everything after the second-to-last cluster
    clusters = []
    for i in idx:
        if clusters and i - clusters[-1][-1] <= 2:
            clusters[-1].append(i)
        else:
            clusters.append([i])
    step = rows[clusters[-2][-1] + 1:clusters[-1][-1] + 1]
    t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
    c, n = collections.Counter(), collections.Counter()
    for r in step:
        k = r["Kernel_Name"].split("(")[0][:100]
        c[k] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        n[k] += 1
    busy = sum(c.values())
    print(f"one step: wall {(t1 - t0) / 1e6:.1f} ms, kernel busy {busy / 1e6:.1f} ms, {len(step)} kernels\n")
    print("| kernel | calls | ms | % |\n|---|---:|---:|---:|")
    for k, v in c.most_common(a.top):
        print(f"| `{k}` | {n[k]} | {v / 1e6:.2f} | {100 * v / busy:.1f} |")


if __name__ == "__main__":
    main()
