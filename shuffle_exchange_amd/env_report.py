"""Environment / native-op report (parity: reference env_report.py, ``ds_report``).

Lists the torch / ROCm / RCCL stack, the visible MI355X devices and, for every native extension,
whether it is built in-tree and loads, plus the ops it registers. There is no JIT op builder
(SURVEY §0): the "compatible / installed" columns of the reference collapse into built + loaded.
"""
import os
import shutil
import subprocess

GREEN, RED, END = "\033[92m", "\033[91m", "\033[0m"


def _ok(b):
    return f"{GREEN}[OKAY]{END}" if b else f"{RED}[NO]{END}"


def native_report():
    from .ops import native
    import torch
    rows = []
    for kind, path in (("hip (gfx950 kernels)", native.HIP_LIB), ("cpu (Adam/Lion/Adagrad, AIO)", native.CPU_LIB)):
        built = os.path.exists(path)
        loaded = False
        if built:
            try:
                torch.ops.load_library(path)
                loaded = True
            except Exception:
                loaded = False
        rows.append((kind, built, loaded, path))
    ops = {}
    for ns in ("sxe", "sxe_cpu"):
        try:
            ops[ns] = sorted(n for n in dir(getattr(torch.ops, ns)) if not n.startswith("_") and n not in
                             ("name", "op", "load_library"))
        except Exception:
            ops[ns] = []
    return rows, ops


def _hipcc_version():
    exe = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    try:
        out = subprocess.run([exe, "--version"], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                             timeout=20).stdout
        return next((l for l in out.splitlines() if "HIP version" in l), out.splitlines()[0] if out else "?")
    except Exception:
        return "not found"


def main(hide_operator_status=False, hide_errors_and_warnings=False):
    import torch
    from . import __version__
    print("-" * 70)
    print("shuffle_exchange_amd environment report")
    print("-" * 70)
    if not hide_operator_status:
        rows, ops = native_report()
        print(f"{'extension':34s} {'built':8s} {'loaded':8s}")
        for kind, built, loaded, path in rows:
            print(f"{kind:34s} {_ok(built):17s} {_ok(loaded)}")
        for ns, names in ops.items():
            print(f"  torch.ops.{ns}: {', '.join(names) if names else '-'}")
    print("-" * 70)
    print(f"torch version ................ {torch.__version__}")
    print(f"torch hip version ............ {getattr(torch.version, 'hip', None)}")
    print(f"hipcc ........................ {_hipcc_version()}")
    try:
        nccl = ".".join(map(str, torch.cuda.nccl.version()))
    except Exception:
        nccl = "n/a"
    print(f"rccl version ................. {nccl}")
    print(f"shuffle_exchange_amd ......... {__version__} ({os.path.dirname(os.path.abspath(__file__))})")
    n = torch.cuda.device_count()
    print(f"visible GPUs ................. {n}")
    if n and torch.cuda.is_available():
        for i in range(n):
            p = torch.cuda.get_device_properties(i)
            arch = getattr(p, "gcnArchName", "?")
            print(f"  [{i}] {p.name} {arch} {p.total_memory / 2**30:.0f} GiB, {p.multi_processor_count} CUs")
    print("-" * 70)


if __name__ == "__main__":
    main()
