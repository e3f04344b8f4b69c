"""Async-I/O throughput benchmark and parameter sweep for ZeRO-Infinity swap folders.

Parity: reference nvme/test_ds_aio.py + ds_aio_args.py (``ds_io``: --folder --io_size --read
--block_size --queue_depth --io_parallel --loops --gpu --validate), perf_run_sweep.py /
perf_generate_param.py (``ds_nvme_tune``: sweep block size x queue depth x parallelism, report the
best and emit the ``aio`` config block). The engine under test is this repo's C++ thread-pool AIO
(csrc/cpu/aio.cpp, O_DIRECT when aligned) reading/writing pinned host buffers; ``--gpu`` adds the
hipMemcpy leg into HBM so the number is the end-to-end swap-in/out rate ZeRO-Infinity sees.
"""
import argparse
import itertools
import json
import os
import time

import torch


def parse_size(s):
    s = str(s).strip().upper()
    mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}
    return int(float(s[:-1]) * mult[s[-1]]) if s[-1] in mult else int(s)


def io_benchmark(folder, io_size, read=False, block_size=1 << 20, queue_depth=32, io_parallel=4, loops=3,
                 gpu=False, validate=False, warmup_loops=1):
    """Returns dict(GB/s, seconds per loop) for one configuration."""
    from ..ops.aio import AsyncIOHandle
    os.makedirs(folder, exist_ok=True)
    path = os.path.join(folder, f"sxe_io_{os.getpid()}.bin")
    h = AsyncIOHandle(block_size=block_size, queue_depth=queue_depth, intra_op_parallelism=io_parallel)
    buf = AsyncIOHandle.new_cpu_locked_tensor(io_size, torch.empty(0, dtype=torch.uint8))
    buf.copy_(torch.randint(0, 255, (io_size,), dtype=torch.uint8))
    dev = torch.empty(io_size, dtype=torch.uint8, device="cuda") if gpu and torch.cuda.is_available() else None
    if read:
        h.sync_pwrite(buf, path, 0)
    times = []
    for i in range(warmup_loops + loops):
        t0 = time.perf_counter()
        if read:
            h.async_pread(buf, path, 0)
            h.wait()
            if dev is not None:
                dev.copy_(buf, non_blocking=True)
                torch.cuda.synchronize()
        else:
            if dev is not None:
                buf.copy_(dev, non_blocking=True)
                torch.cuda.synchronize()
            h.async_pwrite(buf, path, 0)
            h.wait()
        if i >= warmup_loops:
            times.append(time.perf_counter() - t0)
    ok = True
    if validate:
        chk = torch.empty_like(buf)
        h.sync_pread(chk, path, 0)
        ok = bool(torch.equal(chk, buf))
    try:
        os.remove(path)
    except OSError:
        pass
    t = sum(times) / len(times)
    return {"read": read, "io_size": io_size, "block_size": block_size, "queue_depth": queue_depth,
            "io_parallel": io_parallel, "gpu": dev is not None, "GB/s": io_size / t / 1e9, "sec": t, "valid": ok}


def sweep(folder, io_size, block_sizes=(1 << 20, 4 << 20, 16 << 20), queue_depths=(8, 32, 128),
          parallelism=(1, 4, 8), loops=2):
    """Grid over (block size, queue depth, threads) for reads and writes; returns results and the
    best-read ``aio`` config block (reference ds_nvme_tune)."""
    res = []
    for read, bs, qd, par in itertools.product((True, False), block_sizes, queue_depths, parallelism):
        res.append(io_benchmark(folder, io_size, read, bs, qd, par, loops))
    best = max((r for r in res if r["read"]), key=lambda r: r["GB/s"])
    aio = {"block_size": best["block_size"], "queue_depth": best["queue_depth"],
           "intra_op_parallelism": best["io_parallel"], "single_submit": False, "overlap_events": True}
    return res, {"aio": aio}


def main(argv=None):
    ap = argparse.ArgumentParser("sxe_io")
    ap.add_argument("--folder", required=True)
    ap.add_argument("--io_size", default="256M")
    ap.add_argument("--read", action="store_true")
    ap.add_argument("--block_size", default="1M")
    ap.add_argument("--queue_depth", type=int, default=32)
    ap.add_argument("--io_parallel", type=int, default=4)
    ap.add_argument("--loops", type=int, default=3)
    ap.add_argument("--gpu", action="store_true")
    ap.add_argument("--validate", action="store_true")
    ap.add_argument("--sweep", action="store_true", help="ds_nvme_tune: grid search and print the aio config")
    a = ap.parse_args(argv)
    size = parse_size(a.io_size)
    if a.sweep:
        res, cfg = sweep(a.folder, size)
        for r in res:
            print(json.dumps(r))
        print(json.dumps(cfg))
        return cfg
    r = io_benchmark(a.folder, size, a.read, parse_size(a.block_size), a.queue_depth, a.io_parallel, a.loops,
                     a.gpu, a.validate)
    print(json.dumps(r))
    return r


if __name__ == "__main__":
    main()
