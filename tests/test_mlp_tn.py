"""Fused SwiGLU MLP (ops/mlp.py) and its dual-layout gated kernels (csrc/kernels/act.hip).

Numerics are checked against a plain fp32 PyTorch formula of the same op; the engine test checks
that a ZeRO-3 Llama step with the fused MLP matches the module path (SXE_MLP_TN=0 equivalent).
"""
import pytest
import torch
import torch.nn.functional as F

from shuffle_exchange_amd.ops import mlp as mlp_ops
from shuffle_exchange_amd.ops.linear import Linear


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def test_cpu_falls_back_to_module_path():
    torch.manual_seed(0)
    gu, dn = Linear(64, 256, bias=False), Linear(128, 64, bias=False)
    x = torch.randn(2, 64, 64, requires_grad=True)
    assert not mlp_ops.fused_ok(x, gu, dn)
    y = mlp_ops.swiglu_mlp(x, gu, dn)
    g, u = F.linear(x, gu.weight).chunk(2, -1)
    torch.testing.assert_close(y, F.linear(F.silu(g) * u, dn.weight))


@pytest.mark.gpu
@pytest.mark.parametrize("T,I", [(128, 256), (2048, 1536)])
@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4])
def test_dual_gated_kernels_vs_fp32(T, I, variant):
    from shuffle_exchange_amd.ops import native
    native.require_hip()
    torch.manual_seed(0)
    gu = torch.randn(T, 2 * I, device="cuda", dtype=torch.bfloat16)
    d = torch.randn(T, I, device="cuda", dtype=torch.bfloat16)
    h, hT = torch.ops.sxe.gated_act_fwd_dual(gu, 3, variant)
    g, u = gu.float().chunk(2, -1)
    ref = F.silu(g) * u
    assert _rel(h, ref) < 5e-3
    assert torch.equal(hT, h.t())
    dgu, dguT = torch.ops.sxe.gated_act_bwd_dual(d, gu, 3, variant)
    s = torch.sigmoid(g)
    ref_dg = d.float() * u * s * (1 + g * (1 - s))
    ref_du = d.float() * F.silu(g)
    assert _rel(dgu[:, :I], ref_dg) < 5e-3 and _rel(dgu[:, I:], ref_du) < 5e-3
    assert torch.equal(dguT, dgu.t())
    # the token-major outputs equal the existing single-layout kernels bit for bit
    assert torch.equal(h, torch.ops.sxe.gated_act_fwd(gu, 3))
    assert torch.equal(dgu, torch.ops.sxe.gated_act_bwd(d, gu, 3))


@pytest.mark.gpu
def test_fused_mlp_grads_vs_fp32_autograd():
    torch.manual_seed(0)
    H, I, T = 256, 512, 512
    gu = Linear(H, 2 * I, bias=False).cuda().bfloat16()
    dn = Linear(I, H, bias=False).cuda().bfloat16()
    x = torch.randn(2, T // 2, H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    assert mlp_ops.fused_ok(x, gu, dn)
    y = mlp_ops.swiglu_mlp(x, gu, dn)
    dy = torch.randn_like(y)
    y.backward(dy)
    # fp32 reference of the same op
    xr = x.detach().float().requires_grad_()
    wgu = gu.weight.detach().float().requires_grad_()
    wd = dn.weight.detach().float().requires_grad_()
    g, u = F.linear(xr, wgu).chunk(2, -1)
    yr = F.linear(F.silu(g) * u, wd)
    yr.backward(dy.float())
    assert _rel(y, yr) < 1e-2
    assert _rel(x.grad, xr.grad) < 1e-2
    assert _rel(gu.weight.grad, wgu.grad) < 1e-2
    assert _rel(dn.weight.grad, wd.grad) < 1e-2


@pytest.mark.gpu
def test_fused_mlp_writes_zero_grad_targets():
    """With an optimizer-provided fp32 target the weight grads are accumulated there (as ZeRO
    installs them) instead of being returned."""
    torch.manual_seed(0)
    H, I, T = 128, 256, 256
    gu = Linear(H, 2 * I, bias=False).cuda().bfloat16()
    dn = Linear(I, H, bias=False).cuda().bfloat16()
    bufs = {gu.weight: torch.full((2 * I, H), 0.5, device="cuda"), dn.weight: torch.zeros(H, I, device="cuda")}
    done = []
    for w in bufs:
        w._sxe_grad_target = lambda p: (bufs[p], p is gu.weight)  # accumulate into gate_up's buffer only
        w._sxe_grad_done = lambda p: done.append(p)
    x = torch.randn(T, H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    y = mlp_ops.swiglu_mlp(x, gu, dn)
    dy = torch.randn_like(y)
    y.backward(dy)
    assert gu.weight.grad is None and dn.weight.grad is None and len(done) == 2
    g, u = F.linear(x.float(), gu.weight.float()).chunk(2, -1)
    h = F.silu(g) * u
    dwd = dy.float().t() @ h
    dh = dy.float() @ dn.weight.float()
    s = torch.sigmoid(g)
    dgu = torch.cat([dh * u * s * (1 + g * (1 - s)), dh * F.silu(g)], -1)
    dwgu = dgu.t() @ x.float()
    assert _rel(bufs[dn.weight], dwd) < 1e-2
    assert _rel(bufs[gu.weight] - 0.5, dwgu) < 1e-2


@pytest.mark.gpu
def test_llama_zero3_step_fused_mlp_matches_module_path(monkeypatch):
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config

    def run(enabled):
        monkeypatch.setattr(mlp_ops, "ENABLED", enabled)
        torch.manual_seed(0)
        cfg = llama_config("llama-tiny", hidden_size=256, intermediate_size=512, num_attention_heads=2,
                           num_key_value_heads=1, vocab_size=512, num_hidden_layers=2)
        with sxe.zero.Init(dtype=torch.bfloat16):
            model = LlamaForCausalLM(cfg)
        ds = {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": 2, "bf16": {"enabled": True},
              "zero_optimization": {"stage": 3}, "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}}}
        eng, _, _, _ = sxe.initialize(model=model, config=ds)
        g = torch.Generator(device="cuda").manual_seed(5)
        losses = []
        for _ in range(4):
            ids = torch.randint(0, cfg.vocab_size, (2, 128), device="cuda", generator=g)
            loss = eng(ids, labels=ids)
            eng.backward(loss)
            eng.step()
            losses.append(float(loss))
        return losses

    fused, plain = run(True), run(False)
    assert all(abs(a - b) < 2e-2 * abs(b) for a, b in zip(fused, plain)), (fused, plain)
