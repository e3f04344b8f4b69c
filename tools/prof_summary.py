#!/usr/bin/env python3
"""Summarise a rocprofv3 ``*_kernel_stats.csv`` into a compact markdown table (top kernels and
per-category totals) for committing under profiles/.

Usage: python tools/prof_summary.py gpurun_out/prof/bench_kernel_stats.csv --steps 2 \
          --title "Llama-3-8B ZeRO-3 bf16, 1x MI355X" > profiles/bench_r01.md
"""
import argparse
import csv
import re

CATS = [
    ("GEMM (hipBLASLt/Tensile)", r"^(Custom_)?Cijk_|gemm|Gemm"),
    ("flash attention (sxe)", r"sxe::fa::"),
    ("optimizer (sxe)", r"adam|lion|adagrad|sumsq"),
    ("norm (sxe)", r"sxe::norm_"),
    ("activation (sxe)", r"sxe::gated_|sxe::bias_act"),
    ("rope (sxe)", r"sxe::rope"),
    ("cross-entropy (sxe)", r"sxe::xent"),
    ("RCCL", r"ncclDevKernel|ncclKernel|rccl"),
    ("copies/fills", r"copyBuffer|fillBuffer|FillFunctor|copy_kernel|direct_copy"),
    ("embedding", r"embedding|compute_grad_weight|sum_and_scatter|radix_sort|merge|indexSelect|gather"),
    ("random (synthetic data)", r"distribution_"),
]


def short(name, n=90):
    name = re.sub(r"\(.*", "", name)
    return name if len(name) <= n else name[:n - 3] + "..."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=1, help="optimizer steps inside the trace")
    ap.add_argument("--top", type=int, default=20)
    ap.add_argument("--title", default="kernel profile")
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((r["Name"], int(r["Calls"]), int(r["TotalDurationNs"])))
    total = sum(t for _, _, t in rows)
    cats = {c: 0 for c, _ in CATS}
    cats["other elementwise/reduce (torch)"] = 0
    for name, _, t in rows:
        for c, pat in CATS:
            if re.search(pat, name):
                cats[c] += t
                break
        else:
            cats["other elementwise/reduce (torch)"] += t
    print(f"# {a.title}\n")
    print(f"Total GPU kernel time: {total / 1e6:.1f} ms over the trace "
          f"({total / 1e6 / a.steps:.1f} ms per step, {a.steps} step(s) traced incl. warmup if any)\n")
    print("| category | ms | % |\n|---|---:|---:|")
    for c, t in sorted(cats.items(), key=lambda kv: -kv[1]):
        if t:
            print(f"| {c} | {t / 1e6:.1f} | {100 * t / total:.1f} |")
    print(f"\n## Top {a.top} kernels\n")
    print("| kernel | calls | total ms | avg us | % |\n|---|---:|---:|---:|---:|")
    for name, calls, t in sorted(rows, key=lambda r: -r[2])[:a.top]:
        print(f"| `{short(name)}` | {calls} | {t / 1e6:.1f} | {t / calls / 1e3:.1f} | {100 * t / total:.1f} |")


if __name__ == "__main__":
    main()
