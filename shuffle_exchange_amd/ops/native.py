"""Loader for the in-tree native extensions.

``_sxe_hip.so`` holds every gfx950 HIP kernel (registered as ``torch.ops.sxe.*``) and
``_sxe_cpu.so`` the host C++ kernels (CPU Adam family, async I/O engine). Both are built ahead of
time by ``csrc/build.py`` (``__graft_entry__.build()`` runs it); there is no JIT builder.

Policy (MI355X-first, no silent fallbacks):
  * On a GPU process the HIP extension MUST load; ``require_hip()`` raises otherwise, so a
    missing build fails loudly instead of silently running a PyTorch path.
  * On a CPU-only process (the gloo plumbing tests) the ops use their PyTorch reference
    implementations, which are also the numerics oracles for the kernel tests.
"""
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
HIP_LIB = os.environ.get("SXE_HIP_LIB") or os.path.join(_HERE, "_sxe_hip.so")  # override: A/B kernel experiments
CPU_LIB = os.path.join(_HERE, "_sxe_cpu.so")

_lock = threading.Lock()
_state = {"hip": None, "cpu": None, "hip_err": None, "cpu_err": None}


def _load(kind, path):
    # lock-free once decided: the dispatch predicates run inside torch.compile'd regions, and Dynamo
    # cannot enter a lock (a graph break there splits the model into per-layer frames)
    done = _state[kind]
    if done is not None:
        return done
    with _lock:
        if _state[kind] is not None:
            return _state[kind]
        if not os.path.exists(path):
            _state[kind] = False
            _state[kind + "_err"] = f"{path} not built (run `python csrc/build.py`)"
            return False
        try:
            torch.ops.load_library(path)
            _state[kind] = True
        except Exception as e:  # pragma: no cover - depends on the box
            _state[kind] = False
            _state[kind + "_err"] = repr(e)
        return _state[kind]


def hip_available():
    """True when the HIP kernels can be used (extension loaded AND a GPU is present)."""
    return torch.cuda.is_available() and _load("hip", HIP_LIB)


def require_hip():
    if not torch.cuda.is_available():
        raise RuntimeError("sxe: HIP kernels requested on a process without a GPU")
    if not _load("hip", HIP_LIB):
        raise RuntimeError(f"sxe: native HIP extension failed to load: {_state['hip_err']}")
    return torch.ops.sxe


def cpu_available():
    return _load("cpu", CPU_LIB)


def require_cpu():
    if not _load("cpu", CPU_LIB):
        raise RuntimeError(f"sxe: native CPU extension failed to load: {_state['cpu_err']}")
    return torch.ops.sxe_cpu


def use_hip(t):
    """Dispatch predicate for a tensor argument: GPU tensors go to the HIP kernels (and fail
    loudly if those are missing); CPU tensors use the PyTorch reference path."""
    if t.is_cuda:
        require_hip()
        return True
    return False


def status():
    return {"hip": _load("hip", HIP_LIB), "cpu": _load("cpu", CPU_LIB),
            "hip_err": _state["hip_err"], "cpu_err": _state["cpu_err"]}
