#!/usr/bin/env python3
"""Ahead-of-time build of the native extensions (gfx950 HIP kernels + host C++).

Outputs (in-tree, next to the Python loaders so they travel with the repo):
  shuffle_exchange_amd/ops/_sxe_hip.so   all HIP kernels (torch.ops.sxe.*), gfx950 only
  shuffle_exchange_amd/ops/_sxe_cpu.so   host kernels: CPU Adam/Lion/Adagrad (AVX-512/AVX2
                                         runtime dispatch + OpenMP) and the async-IO engine

There is no JIT op_builder (the reference's `op_builder/*` is a per-op JIT):
every extension is compiled once with hipcc / g++ and loaded with torch.ops.load_library.
Incremental: an object is rebuilt only if its source or any header under csrc/include changed.

Usage: python csrc/build.py [-j N] [--force] [--only hip|cpu]
"""
import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
OUT_DIR = os.path.join(ROOT, "shuffle_exchange_amd", "ops")
BUILD_DIR = os.path.join(ROOT, "build", "native")
ARCH = os.environ.get("SXE_OFFLOAD_ARCH", "gfx950")


def _torch_paths():
    import torch
    base = os.path.dirname(torch.__file__)
    inc = [os.path.join(base, "include"), os.path.join(base, "include", "torch", "csrc", "api", "include")]
    lib = os.path.join(base, "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _hash_inputs(src, extra_flags):
    h = hashlib.sha1()
    with open(src, "rb") as f:
        h.update(f.read())
    inc_dir = os.path.join(CSRC, "include")
    for name in sorted(os.listdir(inc_dir)):
        with open(os.path.join(inc_dir, name), "rb") as f:
            h.update(f.read())
    h.update(" ".join(extra_flags).encode())
    return h.hexdigest()


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("command failed:\n  " + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def _compile(kind, src, obj, flags, force):
    stamp = obj + ".sha1"
    digest = _hash_inputs(src, flags)
    if not force and os.path.exists(obj) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read().strip() == digest:
                return obj, False
    compiler = "hipcc" if kind == "hip" else os.environ.get("CXX", "g++")
    _run([compiler] + flags + ["-c", src, "-o", obj])
    with open(stamp, "w") as f:
        f.write(digest)
    return obj, True


def build(jobs=None, force=False, only=None, verbose=True):
    inc, lib, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    os.makedirs(BUILD_DIR, exist_ok=True)
    common = ["-O3", "-fPIC", "-std=c++17", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
              "-DTORCH_API_INCLUDE_EXTENSION_H", "-I" + os.path.join(CSRC, "include"), "-I" + py_inc]
    common += ["-I" + p for p in inc]
    hip_flags = common + [f"--offload-arch={ARCH}", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
                          "-fno-gpu-rdc", "-munsafe-fp-atomics", "-Wno-unused-result",
                          "-Wno-return-type", "-ffp-contract=fast"]
    # -fno-math-errno: std::sqrt in the optimizer loops may not set errno, else GCC keeps them scalar
    cpu_flags = common + ["-fopenmp", "-fno-math-errno", "-Wall", "-Wno-unused-function", "-Wno-sign-compare"]
    targets = []
    if only in (None, "hip"):
        hip_srcs = sorted(f for f in os.listdir(os.path.join(CSRC, "kernels")) if f.endswith(".hip"))
        targets.append(("hip", [os.path.join(CSRC, "kernels", f) for f in hip_srcs],
                        os.path.join(OUT_DIR, "_sxe_hip.so"), hip_flags,
                        ["-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-lamdhip64"]))
    if only in (None, "cpu"):
        cpu_srcs = sorted(f for f in os.listdir(os.path.join(CSRC, "cpu")) if f.endswith(".cpp"))
        targets.append(("cpu", [os.path.join(CSRC, "cpu", f) for f in cpu_srcs],
                        os.path.join(OUT_DIR, "_sxe_cpu.so"), cpu_flags,
                        ["-lc10", "-ltorch", "-ltorch_cpu", "-fopenmp", "-lpthread"]))
    jobs = jobs or min(8, os.cpu_count() or 4)
    results = {}
    with cf.ThreadPoolExecutor(jobs) as ex:
        futs = {}
        for kind, srcs, so, flags, _ in targets:
            for s in srcs:
                obj = os.path.join(BUILD_DIR, kind + "_" + os.path.basename(s) + ".o")
                futs[ex.submit(_compile, kind, s, obj, flags, force)] = (kind, s)
        for fu in cf.as_completed(futs):
            kind, s = futs[fu]
            obj, rebuilt = fu.result()
            results.setdefault(kind, []).append((obj, rebuilt))
            if verbose and rebuilt:
                print(f"[sxe-build] compiled {os.path.relpath(s, ROOT)}", flush=True)
    for kind, srcs, so, flags, libs in targets:
        objs = sorted(o for o, _ in results.get(kind, []))
        relink = force or not os.path.exists(so) or any(r for _, r in results.get(kind, []))
        relink = relink or any(os.path.getmtime(o) > os.path.getmtime(so) for o in objs)
        if relink:
            linker = "hipcc" if kind == "hip" else os.environ.get("CXX", "g++")
            extra = [f"--offload-arch={ARCH}"] if kind == "hip" else []
            _run([linker, "-shared", "-fPIC"] + extra + objs + ["-o", so, "-L" + lib,
                  f"-Wl,-rpath,{lib}"] + libs)
            if verbose:
                print(f"[sxe-build] linked {os.path.relpath(so, ROOT)}", flush=True)
    return [t[2] for t in targets]


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", choices=["hip", "cpu"], default=None)
    a = ap.parse_args()
    try:
        build(a.jobs, a.force, a.only)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
