"""RCCL (backend "nccl") on the GPU box: the comm facade's init path (device-bound
init_process_group, so sub-communicators split from the world comm) in a world of one process, then
every collective the ZeRO / MoE / SP engines issue -- all_reduce, reduce_scatter_tensor,
all_gather_into_tensor, all_to_all_single, broadcast, on a new_group sub-communicator too -- run as
RCCL kernels on that process group (torch.distributed directly: the facade short-cuts a world of one)
and checked against their single-rank results, in bf16 and fp32. Multi-rank RCCL needs one GPU per
rank, so world sizes > 1 are covered by the gloo tests and the driver's multi-GPU runs."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import torch
import torch.distributed as tdist
from shuffle_exchange_amd import comm as dist
dist.init_distributed(dist_backend="nccl", verbose=False)
assert dist.get_backend() == "nccl", dist.get_backend()
dev = torch.device("cuda", 0)
sub = dist.new_group([0])
for grp in (None, sub):
    for dt in (torch.float32, torch.bfloat16):
        x = torch.randn(1 << 20, device=dev, dtype=dt)
        y = x.clone()
        tdist.all_reduce(y, group=grp)
        assert torch.equal(y, x)
        out = torch.empty_like(x)
        tdist.reduce_scatter_tensor(out, x, group=grp)
        assert torch.equal(out, x)
        g = torch.empty_like(x)
        tdist.all_gather_into_tensor(g, x, group=grp)
        assert torch.equal(g, x)
        a2a = torch.empty_like(x)
        tdist.all_to_all_single(a2a, x, group=grp)
        assert torch.equal(a2a, x)
        b = x.clone()
        tdist.broadcast(b, 0, group=grp)
        assert torch.equal(b, x)
# the facade on the same group (world of one: local copies, no collective launched)
bf = torch.randn(4096, device=dev, dtype=torch.bfloat16)
o2 = torch.empty_like(bf)
dist.reduce_scatter_tensor(o2, bf)
assert torch.equal(o2, bf)
torch.cuda.synchronize()
dist.barrier()
print("RCCL_OK", torch.cuda.nccl.version() if hasattr(torch.cuda, "nccl") else "")
dist.destroy_process_group()
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_world_of_one_collectives():
    env = dict(os.environ, PYTHONPATH=ROOT, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    env.pop("SXE_DIST_BACKEND", None)
    r = subprocess.run([sys.executable, "-c", SCRIPT], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0 and "RCCL_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])
