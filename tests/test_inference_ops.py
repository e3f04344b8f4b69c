"""Functional inference-v1 ops (ops/inference_ops.py) against their PyTorch formulas (CPU)."""
import torch
import torch.nn.functional as F

from shuffle_exchange_amd.ops import inference_ops as io


def test_norms_bias_and_residual_ops():
    torch.manual_seed(0)
    x, r = torch.randn(3, 5, 64), torch.randn(3, 5, 64)
    g, b = torch.rand(64) + 0.5, torch.randn(64)
    torch.testing.assert_close(io.layer_norm(x, g, b, 1e-5), F.layer_norm(x, (64,), g, b, 1e-5), atol=1e-5, rtol=1e-5)
    rms = lambda t: t * torch.rsqrt(t.pow(2).mean(-1, keepdim=True) + 1e-6) * g  # noqa: E731
    torch.testing.assert_close(io.rms_norm(x, g, 1e-6), rms(x), atol=1e-5, rtol=1e-5)
    y, h = io.pre_rms_norm(x, r, g, 1e-6)
    torch.testing.assert_close(h, x + r)
    torch.testing.assert_close(y, rms(x + r), atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(io.bias_add(x, b), x + b)
    torch.testing.assert_close(io.bias_gelu(x, b), F.gelu(x + b, approximate="tanh"), atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(io.bias_relu(x, b), F.relu(x + b))
    torch.testing.assert_close(io.bias_residual(x, r, b), x + r + b)
    torch.testing.assert_close(io.vector_add(x, r, 0.5), x + 0.5 * r)
    gu = torch.randn(3, 128)
    gb = torch.randn(128)
    ref = F.silu((gu + gb)[:, :64]) * (gu + gb)[:, 64:]
    torch.testing.assert_close(io.gated_activation(gu, gb, "GATED_SILU"), ref, atol=1e-5, rtol=1e-5)


def test_gemm_ops():
    torch.manual_seed(1)
    x, r = torch.randn(2, 4, 32), torch.randn(2, 4, 32)
    W = torch.randn(32, 96)  # [in, out]
    g, b = torch.rand(32) + 0.5, torch.randn(32)
    out, norm = io.qkv_gemm(x, W, torch.randn(96) * 0, g, b, 1e-5)
    torch.testing.assert_close(norm, F.layer_norm(x, (32,), g, b, 1e-5), atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(out, norm @ W, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(io.vector_matmul(x, W), x @ W, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(io.linear(x, W.t().contiguous(), None, transposed_mode=True), x @ W, atol=1e-4,
                               rtol=1e-4)
    W1, W2, b1 = torch.randn(32, 64), torch.randn(64, 32), torch.randn(64)
    o, h = io.mlp_gemm(x, r, W1, W2, None, b1, g, b, 1e-5, act="relu")
    torch.testing.assert_close(h, x + r)
    ref = F.relu(F.layer_norm(x + r, (32,), g, b, 1e-5) @ W1 + b1) @ W2
    torch.testing.assert_close(o, ref, atol=1e-4, rtol=1e-4)


def test_softmax_and_context_with_cache():
    torch.manual_seed(2)
    s = torch.randn(1, 2, 3, 5)
    p = io.softmax(s, None, triangular=True)
    mask = torch.arange(5)[None, :] > torch.arange(2, 5)[:, None]
    torch.testing.assert_close(p, torch.softmax(s.masked_fill(mask, float("-inf")), -1))
    # incremental decoding == one-shot causal attention over the full sequence
    H, KV, D = 4, 2, 8
    qkv = torch.randn(1, 6, (H + 2 * KV) * D)
    ws = io.Workspace()
    full, _, _ = io.softmax_context(qkv, None, H, KV, D ** 0.5, layer_id=0, rotary_dim=4, workspace=ws)
    ws2 = io.Workspace()
    a, _, _ = io.softmax_context(qkv[:, :4], None, H, KV, D ** 0.5, layer_id=0, rotary_dim=4, workspace=ws2)
    b2, k, _ = io.softmax_context(qkv[:, 4:], None, H, KV, D ** 0.5, layer_id=0, rotary_dim=4, workspace=ws2)
    assert k.shape[1] == 6
    torch.testing.assert_close(torch.cat([a, b2], 1), full, atol=1e-5, rtol=1e-5)


def test_moe_and_layout_ops():
    torch.manual_seed(3)
    res, out, coef = torch.randn(4, 8), torch.randn(4, 8), torch.softmax(torch.randn(4, 2), -1)
    torch.testing.assert_close(io.moe_res_matmul(res, coef, out), res * coef[:, :1] + out * coef[:, 1:])
    Q, W = torch.rand(5, 3, 2), torch.randn(5, 7)
    torch.testing.assert_close(io.einsum_sec_sm_ecm(Q, W), torch.einsum("sec,sm->ecm", Q, W))
    q = torch.randn(2, 3, 4 * 20)
    pq, pk, pv = io.pad_transform(q, q, q, 4)
    assert pq.shape == (2, 4, 3, 32) and torch.equal(pq[..., :20], q.view(2, 3, 4, 20).transpose(1, 2))
