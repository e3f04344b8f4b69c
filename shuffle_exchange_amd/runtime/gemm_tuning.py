"""Per-shape GEMM solution selection for MI355X (hipBLASLt / rocBLAS) via PyTorch TunableOp.

The plain library GEMMs (projections, LM head) are ~75 % of a Llama training step. hipBLASLt's
default heuristic is not always its fastest solution for a given (M, N, K, layout); TunableOp
benchmarks all candidate solutions once per shape on the target GPU and records the winner.
``tools/tune_gemms.py`` produces the table on an MI355X; the framework ships it
(``tuning/tunableop_mi355x.csv``) and loads it read-only at engine start, so training runs never
pay tuning time. Entries are validated by PyTorch against the GPU arch / ROCm / hipBLASLt versions
and ignored on mismatch.
"""
import os

import torch

from ..utils.logging import log_dist

PACKAGED = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning",
                        "tunableop_mi355x.csv")
_loaded = {"path": None}


def load_tuned_gemms(path=None):
    """Enable TunableOp in lookup-only mode with the given (or packaged) results file."""
    if not torch.cuda.is_available() or os.environ.get("SXE_GEMM_TUNING", "1") == "0":
        return False
    path = path or os.environ.get("SXE_TUNABLEOP_FILE") or PACKAGED
    if not path or not os.path.exists(path):
        return False
    if _loaded["path"] == path:
        return True
    tun = torch.cuda.tunable
    tun.enable(True)
    # SXE_GEMM_TUNE_OUT=<csv>: tune the shapes this run meets that the table lacks (bounded search per
    # shape) and write the table there -- merge it into the packaged file with tools/merge_tunableop.py
    out = os.environ.get("SXE_GEMM_TUNE_OUT")
    tun.tuning_enable(bool(out))
    if out:
        tun.set_filename(out)
        tun.set_max_tuning_duration(int(os.environ.get("SXE_GEMM_TUNE_MS", "200")))
    # the table must have LF line endings: with CRLF the last validator's value carries a '\r'
    # and TunableOp rejects the whole file ("Failed validator: ROCBLAS_VERSION")
    ok = tun.read_file(path)
    if not ok:
        have = dict(tun.get_validators())
        log_dist(f"GEMM tuning table rejected by TunableOp validators (runtime: {have})", ranks=[0])
    _loaded["path"] = path
    log_dist(f"GEMM tuning table loaded: {path} (ok={ok})", ranks=[0])
    return True
