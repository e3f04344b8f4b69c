"""Ragged grouped expert GEMM (csrc/kernels/grouped_gemm.hip, ops/moe.grouped_gemm) vs a plain
fp32 PyTorch per-expert loop; and the dropless MoE of the v2 HF decoder through it."""
import pytest
import torch
import torch.nn.functional as F

from shuffle_exchange_amd.ops import moe as moe_ops


def _ref(x, w, offs, scale=None):
    y = torch.zeros(x.shape[0], w.shape[1], dtype=torch.float32, device=x.device)
    o = offs.tolist()
    for e in range(w.shape[0]):
        y[o[e]:o[e + 1]] = x[o[e]:o[e + 1]].float() @ w[e].float().t()
    if scale is not None:
        y = y * scale.float().view(-1, 1)
    return y


def test_expert_loop_dispatch_rule(monkeypatch):
    """Few experts with >= GG_LOOP_MIN_ROWS rows each -> the per-expert GEMM loop; many small
    experts -> the ragged kernel; the env knob forces either."""
    x = torch.empty(8 * moe_ops.GG_LOOP_MIN_ROWS, 16)
    assert moe_ops._use_expert_loop(x, torch.empty(8, 4, 16))
    assert not moe_ops._use_expert_loop(x, torch.empty(60, 4, 16))
    monkeypatch.setenv("SXE_GG_DISPATCH", "kernel")
    assert not moe_ops._use_expert_loop(x, torch.empty(8, 4, 16))
    monkeypatch.setenv("SXE_GG_DISPATCH", "loop")
    assert moe_ops._use_expert_loop(x[:1], torch.empty(60, 4, 16))


def test_expert_offsets_and_cpu_fallback():
    torch.manual_seed(0)
    flat = torch.tensor([2, 0, 2, 3, 0, 2])
    offs = moe_ops.expert_offsets(flat.sort().values, 5)
    assert offs.tolist() == [0, 2, 2, 5, 6, 6]
    x, w = torch.randn(6, 16), torch.randn(5, 8, 16)
    s = torch.rand(6)
    torch.testing.assert_close(moe_ops.grouped_gemm(x, w, offs, s), _ref(x, w, offs, s))


@pytest.mark.gpu
@pytest.mark.parametrize("dispatch", ["kernel", "loop"])
@pytest.mark.parametrize("counts", [[0, 300, 1, 128, 0, 77, 513, 2], [1], [0, 0, 0, 5]])
@pytest.mark.parametrize("scale", [None, "fp32", "bf16"])
def test_grouped_gemm_vs_fp32(counts, scale, dispatch, monkeypatch):
    monkeypatch.setenv("SXE_GG_DISPATCH", dispatch)
    from shuffle_exchange_amd.ops import native
    native.require_hip()
    torch.manual_seed(0)
    E, N, K = len(counts), 384, 256
    R = sum(counts)
    x = torch.randn(R, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(E, N, K, device="cuda", dtype=torch.bfloat16) / 16
    offs = torch.tensor([0] + list(torch.tensor(counts).cumsum(0)), dtype=torch.int32, device="cuda")
    s = None
    if scale:
        s = torch.rand(R, device="cuda", dtype=torch.float32 if scale == "fp32" else torch.bfloat16)
    y = moe_ops.grouped_gemm(x, w, offs, s)
    ref = _ref(x, w, offs, s)
    assert y.dtype == torch.bfloat16 and y.shape == (R, N)
    err = ((y.float() - ref).norm() / ref.norm()).item()
    assert err < 1e-2, err


@pytest.mark.gpu
def test_dropless_moe_grouped_matches_loop(monkeypatch):
    from shuffle_exchange_amd.inference.v2.model_implementations import hf_decoder
    torch.manual_seed(0)
    T, H, I, E, k = 200, 256, 384, 8, 2
    x = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
    router = torch.randn(E, H, device="cuda", dtype=torch.bfloat16)
    e_gu = torch.randn(E, 2 * I, H, device="cuda", dtype=torch.bfloat16) / 16
    e_down = torch.randn(E, H, I, device="cuda", dtype=torch.bfloat16) / 16
    grouped = hf_decoder.dropless_moe(x, router, e_gu, e_down, k, True)
    monkeypatch.setattr(moe_ops, "grouped_gemm_ok", lambda *a: False)
    loop = hf_decoder.dropless_moe(x, router, e_gu, e_down, k, True)
    err = ((grouped.float() - loop.float()).norm() / loop.float().norm()).item()
    assert err < 2e-2, err
