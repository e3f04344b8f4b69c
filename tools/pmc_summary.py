"""Summarise rocprofv3 --pmc counter_collection.csv files (one per pass) into a markdown table of
per-kernel mean counter values plus derived ratios.
  python tools/pmc_summary.py gpurun_out/pmc/pass*/ > profiles/pmc_kernels.md"""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name):
    n = name.split("(")[0]
    for pre in ("void ", "sxe::"):
        n = n.replace(pre, "")
    return n[:60]


def main():
    vals = defaultdict(lambda: defaultdict(list))
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                name = r.get("Kernel_Name") or r.get("Kernel-Name") or r.get("KernelName") or ""
                cn = r.get("Counter_Name") or r.get("Counter-Name")
                cv = r.get("Counter_Value") or r.get("Counter-Value")
                if name and cn and cv:
                    vals[short(name)][cn].append(float(cv))
    keep = [k for k in vals if any(s in k for s in ("fa::", "mx_gemm", "skinny", "paged_attn", "norm_fwd", "adam", "wgrad", "Cijk", "gated_dual", "grouped_gemm", "xent", "acc2", "transpose16"))]
    cols = sorted({c for k in keep for c in vals[k]})
    print("| kernel | " + " | ".join(cols) + " | derived |")
    print("|---|" + "---:|" * len(cols) + "---|")
    for k in sorted(keep):
        m = {c: (sum(v) / len(v)) for c, v in vals[k].items()}
        der = []
        if m.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs, MFMA busy over the 1024 SIMDs (256 CUs x 4)
            util = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 1024)
            der.append(f"MFMA busy {100 * util:.0f} %")
        if m.get("SQ_INSTS_LDS") and "SQ_LDS_BANK_CONFLICT" in m:
            der.append(f"LDS conflict cycles/LDS instr {m['SQ_LDS_BANK_CONFLICT'] / m['SQ_INSTS_LDS']:.3f}")
        if "SQ_INSTS_VALU_MFMA_MOPS_BF16" in m:
            der.append(f"BF16 MFMA GFLOP {m['SQ_INSTS_VALU_MFMA_MOPS_BF16'] * 512 / 1e9:.1f}")
        if "FETCH_SIZE" in m:
            der.append(f"HBM read {m['FETCH_SIZE'] / 1e6:.3f} GB")
        if "WRITE_SIZE" in m:
            der.append(f"HBM write {m['WRITE_SIZE'] / 1e6:.3f} GB")
        print(f"| `{k}` | " + " | ".join(f"{m.get(c, float('nan')):.4g}" for c in cols) + " | " + "; ".join(der) + " |")


if __name__ == "__main__":
    main()
