"""FusedLamb: per-parameter trust ratios (reference ops/lamb/fused_lamb.py:14). Under ZeRO the flat
partitions run the two-stage LAMB with segment tables and an all-reduce of the per-parameter norms,
so a parameter split across ranks gets its WHOLE norm -- ZeRO-1/2/3 on gloo == single-process
FusedLamb over the original parameters."""
import pytest
import torch

from . import _dist_cases as C
from .dist_utils import run_dist

LAMB = {"type": "Lamb", "params": {"lr": 2e-3, "weight_decay": 0.01, "max_coeff": 10.0, "min_coeff": 0.01}}


def _reference(steps, world, mbs, seq):
    from shuffle_exchange_amd.ops.optim import FusedLamb
    model, cfg = C.tiny_llama(0)
    opt = FusedLamb(model.parameters(), lr=2e-3, weight_decay=0.01, max_coeff=10.0, min_coeff=0.01)
    for b in C.global_batches(cfg, world, mbs, seq, steps):
        loss = model(b, labels=b)
        opt.zero_grad()
        loss.backward()
        opt.step()
    return {n: p.detach().float().clone() for n, p in model.named_parameters()}


@pytest.mark.parametrize("stage", [1, 2, 3])
def test_zero_lamb_matches_single_process(stage):
    ds = {"train_micro_batch_size_per_gpu": 2, "optimizer": LAMB,
          "zero_optimization": {"stage": stage, "stage3_param_persistence_threshold": 0}}
    res = run_dist(C.case_train, 2, ds, 3, 2, 16)
    ref = _reference(3, 2, 2, 16)
    for r in res:
        for k, v in ref.items():
            d = (r["params"][k] - v).abs().max().item()
            assert d <= 2e-4 * max(1.0, v.abs().max().item()), (k, d)


def test_lamb_flat_segments_cpu_path():
    """lamb_flat_ over a flat with 3 segments == FusedLamb over the 3 tensors (CPU reference path)."""
    from shuffle_exchange_amd.ops.optim import FusedLamb, lamb_block_table, lamb_flat_
    torch.manual_seed(0)
    shapes = [(37,), (20, 9), (5000,)]
    ps = [torch.randn(s) for s in shapes]
    gs = [torch.randn(s) for s in shapes]
    ref = [torch.nn.Parameter(p.clone()) for p in ps]
    for r, g in zip(ref, gs):
        r.grad = g.clone()
    opt = FusedLamb(ref, lr=1e-2, weight_decay=0.1)
    opt.step()
    flat = torch.cat([p.reshape(-1) for p in ps])
    g = torch.cat([x.reshape(-1) for x in gs])
    m, v = torch.zeros_like(flat), torch.zeros_like(flat)
    segs, off = [], 0
    for i, p in enumerate(ps):
        segs.append((i, off, p.numel()))
        off += p.numel()
    lamb_flat_(flat, g, m, v, None, lamb_block_table(segs, "cpu"), 3, lr=1e-2, beta1=0.9, beta2=0.999, eps=1e-8,
               weight_decay=0.1, step=1)
    assert torch.allclose(flat, torch.cat([r.detach().reshape(-1) for r in ref]), atol=1e-6)
