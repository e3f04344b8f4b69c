"""bench.py driver contract, rehearsed on the CPU: two ranks under torch.distributed.run (gloo),
tiny Llama, one JSON line from rank 0 with the required keys and whole-job token accounting."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_cpu(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", "29631", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--model", "llama-tiny", "--device", "cpu", "--seq", "64", "--mbs", "2", "--gas", "2"]
    r = subprocess.run(cmd, cwd=tmp_path, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-4000:]
    out = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in out, k
    assert out["n_gpus"] == 2 and out["steps"] == 2 and out["warmup"] == 1
    assert out["config"]["global_batch"] == 2 * 2 * 2 and out["config"]["seq_len"] == 64
    tokens = 2 * 2 * 2 * 64 * 2
    assert abs(out["value"] - tokens / (out["ms_per_step"] * 2 / 1000.0)) / out["value"] < 0.01
    assert out["valid_for_metric"] is False  # tiny model on CPU is never a metric number
