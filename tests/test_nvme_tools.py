"""Async-I/O benchmark / sweep tooling (reference deepspeed/nvme ds_io, ds_nvme_tune) on a temp dir."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_io_benchmark_and_sweep(tmp_path):
    from shuffle_exchange_amd.nvme import io_benchmark, parse_size, sweep
    assert parse_size("4M") == 4 << 20 and parse_size("1G") == 1 << 30
    w = io_benchmark(str(tmp_path), 4 << 20, read=False, validate=True, loops=1)
    r = io_benchmark(str(tmp_path), 4 << 20, read=True, validate=True, loops=1)
    assert w["valid"] and r["valid"] and w["GB/s"] > 0 and r["GB/s"] > 0
    res, cfg = sweep(str(tmp_path), 1 << 20, block_sizes=(256 << 10, 1 << 20), queue_depths=(8,),
                     parallelism=(1, 2), loops=1)
    assert len(res) == 8 and set(cfg["aio"]) >= {"block_size", "queue_depth", "intra_op_parallelism"}


def test_sxe_io_cli(tmp_path):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bin", "sxe_io"), "--folder", str(tmp_path),
                          "--io_size", "2M", "--read", "--validate", "--loops", "1"],
                         stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=120)
    assert out.returncode == 0, out.stdout
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["read"] and r["valid"]
