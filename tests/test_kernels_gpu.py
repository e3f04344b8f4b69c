"""Numerics of every HIP kernel vs a plain PyTorch fp32 reference of the same op (MI355X only)."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _native():
    from shuffle_exchange_amd.ops import native
    native.require_hip()


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("gdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("adamw", [True, False])
def test_adam_flat(gdt, adamw):
    from shuffle_exchange_amd.ops.optim import adam_flat_
    n = 1_000_003
    p = torch.randn(n, device="cuda")
    g = torch.randn(n, device="cuda").to(gdt)
    m = torch.randn(n, device="cuda").abs() * 0.1
    v = torch.rand(n, device="cuda") * 0.01
    lp = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    ref = [t.clone().float() for t in (p, g, m, v)]
    scale = torch.tensor([0.5], device="cuda")
    adam_flat_(p, g, m, v, lp, lr=1e-3, beta1=0.9, beta2=0.95, eps=1e-8, weight_decay=0.1, step=3, adamw=adamw,
               scale_t=scale)
    rp, rg, rm, rv = ref
    rg = rg * 0.5
    if not adamw:
        rg = rg + 0.1 * rp
    rm = 0.9 * rm + 0.1 * rg
    rv = 0.95 * rv + 0.05 * rg * rg
    denom = rv.sqrt() / math.sqrt(1 - 0.95 ** 3) + 1e-8
    if adamw:
        rp = rp * (1 - 1e-3 * 0.1)
    rp = rp - (1e-3 / (1 - 0.9 ** 3)) * rm / denom
    assert _rel(p, rp) < 1e-6
    assert _rel(m, rm) < 1e-6 and _rel(v, rv) < 1e-6
    assert torch.equal(lp, p.to(torch.bfloat16))


def test_adam_skip_flag():
    from shuffle_exchange_amd.ops.optim import adam_flat_
    p = torch.randn(4096, device="cuda")
    p0 = p.clone()
    g, m, v = torch.randn_like(p), torch.zeros_like(p), torch.zeros_like(p)
    adam_flat_(p, g, m, v, lr=1.0, skip_t=torch.ones(1, device="cuda"))
    assert torch.equal(p, p0)


def test_multi_tensor_adam_matches_flat():
    from shuffle_exchange_amd.ops.optim import FusedAdam
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(s, device="cuda")) for s in (17, 4096, 70001, 3)]
    ref = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    for p, r in zip(ps, ref):
        p.grad = torch.randn_like(p)
        r.grad = p.grad.clone()
    opt = FusedAdam(ps, lr=1e-2, weight_decay=0.01)
    ropt = torch.optim.AdamW(ref, lr=1e-2, weight_decay=0.01)
    for _ in range(3):
        opt.step()
        ropt.step()
    for p, r in zip(ps, ref):
        assert _rel(p, r) < 1e-5


@pytest.mark.parametrize("H", [128, 1000, 4096, 8192])
@pytest.mark.parametrize("residual", [False, True])
@pytest.mark.parametrize("rows", [1, 185, 300])  # <= 256 rows and H >= 1024: block-per-row forward
def test_rmsnorm(H, residual, rows):
    from shuffle_exchange_amd.ops.norm import rms_norm
    H = H - H % 8
    x = torch.randn(rows, 1, H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn_like(x, requires_grad=True) if residual else None
    w = (torch.rand(H, device="cuda") + 0.5).to(torch.bfloat16).requires_grad_()
    out = rms_norm(x, w, 1e-5, residual=r)
    y, h = (out if residual else (out, None))
    xf = x.float() + (r.float() if residual else 0)
    yr = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5) * w.float()
    assert _rel(y, yr) < 1e-2
    dy = torch.randn_like(y)
    loss = (y.float() * dy.float()).sum() + ((h.float() * 0.5).sum() if residual else 0)
    loss.backward()
    x2 = x.detach().float().requires_grad_()
    r2 = r.detach().float().requires_grad_() if residual else None
    w2 = w.detach().float().requires_grad_()
    xf2 = x2 + (r2 if residual else 0)
    y2 = xf2 * torch.rsqrt(xf2.pow(2).mean(-1, keepdim=True) + 1e-5) * w2
    l2 = (y2 * dy.float()).sum() + ((xf2 * 0.5).sum() if residual else 0)
    l2.backward()
    assert _rel(x.grad, x2.grad) < 2e-2
    assert _rel(w.grad, w2.grad) < 2e-2
    if residual:
        assert _rel(r.grad, r2.grad) < 2e-2


@pytest.mark.parametrize("H", [768, 1024])
def test_layernorm(H):
    from shuffle_exchange_amd.ops.norm import layer_norm
    x = torch.randn(64, H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = (torch.rand(H, device="cuda") + 0.5).to(torch.bfloat16).requires_grad_()
    b = torch.randn(H, device="cuda").to(torch.bfloat16).requires_grad_()
    y = layer_norm(x, w, b, 1e-5)
    x2, w2, b2 = (t.detach().float().requires_grad_() for t in (x, w, b))
    y2 = F.layer_norm(x2, (H,), w2, b2, 1e-5)
    assert _rel(y, y2) < 1e-2
    dy = torch.randn_like(y2)
    (y.float() * dy).sum().backward()
    (y2 * dy).sum().backward()
    for a, c in ((x, x2), (w, w2), (b, b2)):
        assert _rel(a.grad, c.grad) < 2e-2


def test_rope_qkv_roundtrip():
    from shuffle_exchange_amd.ops.rope import RopeCache, _ref_rope, apply_rope_qkv_
    B, S, Hq, Hk, D = 2, 64, 8, 2, 128
    cache = RopeCache(D, 256, 500000.0, device="cuda")
    qkv = torch.randn(B, S, Hq + 2 * Hk, D, device="cuda", dtype=torch.bfloat16)
    ref = qkv.clone().float()
    pos = torch.arange(S, device="cuda").repeat(B)
    rot = _ref_rope(ref[:, :, :Hq + Hk].reshape(B * S, Hq + Hk, D), cache.cos, cache.sin, pos).view(B, S, Hq + Hk, D)
    x = qkv.clone().requires_grad_()
    out = apply_rope_qkv_(x.clone(), cache, Hq + Hk)
    assert _rel(out[:, :, :Hq + Hk], rot) < 1e-2
    assert torch.equal(out[:, :, Hq + Hk:], qkv[:, :, Hq + Hk:])
    g = torch.randn_like(out)
    out.backward(g)
    # backward of an orthogonal rotation = inverse rotation of the gradient
    gi = _ref_rope(g[:, :, :Hq + Hk].float().reshape(B * S, Hq + Hk, D), cache.cos, -cache.sin, pos)
    assert _rel(x.grad[:, :, :Hq + Hk].reshape(B * S, Hq + Hk, D), gi) < 1e-2


@pytest.mark.parametrize("rows", [1, 33])
def test_swiglu(rows):
    from shuffle_exchange_amd.ops.activation import swiglu
    gu = torch.randn(rows, 2 * 1024, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    y = swiglu(gu)
    gu2 = gu.detach().float().requires_grad_()
    g, u = gu2.chunk(2, -1)
    y2 = F.silu(g) * u
    assert _rel(y, y2) < 1e-2
    d = torch.randn_like(y2)
    (y.float() * d).sum().backward()
    (y2 * d).sum().backward()
    assert _rel(gu.grad, gu2.grad) < 2e-2


def test_bias_gelu():
    from shuffle_exchange_amd.ops.activation import bias_gelu
    x = torch.randn(65, 3072, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    b = torch.randn(3072, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    y = bias_gelu(x, b)
    x2, b2 = x.detach().float().requires_grad_(), b.detach().float().requires_grad_()
    y2 = F.gelu(x2 + b2, approximate="tanh")
    assert _rel(y, y2) < 1e-2
    d = torch.randn_like(y2)
    (y.float() * d).sum().backward()
    (y2 * d).sum().backward()
    assert _rel(x.grad, x2.grad) < 2e-2 and _rel(b.grad, b2.grad) < 2e-2


@pytest.mark.parametrize("V", [50257, 128256])
def test_cross_entropy(V):
    from shuffle_exchange_amd.ops.cross_entropy import cross_entropy
    logits = (torch.randn(67, V, device="cuda") * 3).to(torch.bfloat16).requires_grad_()
    tgt = torch.randint(0, V, (67,), device="cuda")
    tgt[5] = -100
    loss = cross_entropy(logits, tgt)
    l2 = logits.detach().float().requires_grad_()
    ref = F.cross_entropy(l2, tgt, ignore_index=-100)
    assert abs(loss.item() - ref.item()) < 1e-2 * abs(ref.item())
    loss.backward()
    ref.backward()
    assert _rel(logits.grad, l2.grad) < 2e-2


def test_fused_linear_cross_entropy():
    from shuffle_exchange_amd.ops.cross_entropy import fused_linear_cross_entropy
    T, H, V = 300, 256, 4096
    h = (torch.randn(T, H, device="cuda") * 0.5).to(torch.bfloat16).requires_grad_()
    W = (torch.randn(V, H, device="cuda") * 0.05).to(torch.bfloat16).requires_grad_()
    tgt = torch.randint(0, V, (T,), device="cuda")
    tgt[:7] = -100
    for chunk in (None, 128):
        h.grad, W.grad = None, None
        loss = fused_linear_cross_entropy(h, W, tgt, chunk_tokens=chunk)
        (loss * 2.0).backward()
        h2, W2 = h.detach().float().requires_grad_(), W.detach().float().requires_grad_()
        ref = F.cross_entropy(h2 @ W2.t(), tgt, ignore_index=-100)
        (ref * 2.0).backward()
        assert abs(loss.item() - ref.item()) < 1e-2 * abs(ref.item())
        assert _rel(h.grad, h2.grad) < 3e-2 and _rel(W.grad, W2.grad) < 3e-2


def test_sumsq():
    from shuffle_exchange_amd.ops.optim import sumsq
    x = torch.randn(3_000_001, device="cuda")
    assert abs(sumsq(x).item() - x.double().pow(2).sum().item()) < 1e-3 * x.double().pow(2).sum().item()
    x[7] = float("inf")
    assert not math.isfinite(sumsq(x).item())


def test_onebit_pack_unpack():
    n = 8 * 100003
    x = torch.randn(n, device="cuda")
    err = torch.empty_like(x)
    scale = (x.norm() / n ** 0.5).reshape(1)
    packed = torch.empty(n // 8, dtype=torch.uint8, device="cuda")
    torch.ops.sxe.sign_pack_ef_(x, err, scale, packed)
    bits = ((packed.cpu().to(torch.int32).unsqueeze(-1) >> torch.arange(8)) & 1).view(-1)
    assert torch.equal(bits.bool(), (x >= 0).cpu())
    dec = torch.where(x >= 0, scale, -scale)
    assert torch.allclose(err, x - dec, atol=1e-6)
    W = 3
    pk = torch.stack([packed, packed ^ 0xFF, packed])
    sc = torch.tensor([1.0, 2.0, 0.5], device="cuda")
    out = torch.empty(n, device="cuda")
    torch.ops.sxe.unpack_avg(pk, sc, out)
    s = (x >= 0).float() * 2 - 1
    ref = (s * 1.0 - s * 2.0 + s * 0.5) / W
    assert torch.allclose(out, ref, atol=1e-6)


@pytest.mark.parametrize("bits", [8, 4])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_quantize_sym(bits, dt):
    from shuffle_exchange_amd.ops import quantizer as Q
    x = torch.randn(128 * 1001, device="cuda").to(dt)
    q, s = Q.quantize(x, 128, bits)
    rq, rs = Q._ref_quant(x.cpu(), 128, bits)
    assert torch.allclose(s.cpu(), rs, rtol=1e-6)
    if bits == 8:  # rounding ties may differ by one step
        assert (q.cpu().view(torch.int8).to(torch.int32) - rq.view(torch.int8).to(torch.int32)).abs().max() <= 1
    out = Q.dequantize(q, s, 128, bits, out=torch.empty_like(x))
    ref = Q._ref_dequant(q.cpu(), s.cpu(), 128, bits, x.numel(), torch.float32)
    assert torch.allclose(out.float().cpu(), ref, atol=1e-2 if dt == torch.bfloat16 else 1e-6)
    err = (out.float() - x.float()).abs().max() / x.float().abs().max()
    assert err < (0.01 if bits == 8 else 0.15)


def test_dequant_reduce():
    from shuffle_exchange_amd.ops import quantizer as Q
    W, m = 4, 128 * 50
    xs = [torch.randn(m, device="cuda") for _ in range(W)]
    qs, ss = zip(*[Q.quantize(x, 128, 8) for x in xs])
    out = torch.zeros(m, device="cuda")
    Q.dequant_reduce(torch.cat(qs), torch.cat(ss), W, 128, 8, out, alpha=0.25)
    ref = sum(Q.dequantize(q, s, 128, 8, out=torch.empty(m, device="cuda")) for q, s in zip(qs, ss)) * 0.25
    assert torch.allclose(out, ref, atol=1e-5)


def test_fp8_quantize():
    from shuffle_exchange_amd.ops import quantizer as Q
    x = torch.randn(512 * 300, device="cuda", dtype=torch.bfloat16) * 3
    q, s = Q.quantize_fp8(x, 512)
    rq, rs = Q.quantize_fp8(x.cpu(), 512)
    assert torch.allclose(s.cpu(), rs, rtol=1e-5)
    out = Q.dequantize_fp8(q, s, 512)
    ref = Q.dequantize_fp8(rq, rs, 512)
    assert ((out.float().cpu() - ref.float()).abs() > 1e-2 * ref.float().abs().clamp_min(1e-3)).float().mean() < 0.01
    assert ((out.float() - x.float()).norm() / x.float().norm()) < 0.05


@pytest.mark.parametrize("variant", [0, 1, 2, 16 * 4])
@pytest.mark.parametrize("K,M,N", [(128, 256, 256), (1024, 768, 512), (2048, 512, 1280)])
@pytest.mark.parametrize("accumulate", [True, False])
def test_wgrad_gemm_vs_fp32_reference(variant, K, M, N, accumulate):
    """Hand-written k-major weight-gradient GEMM (gemm_wgrad.hip, every schedule variant and a
    non-default block order) == fp32 reference of C (+)= alpha * A^T B."""
    g = torch.Generator(device="cuda").manual_seed(K + M + N)
    a = torch.randn(K, M, device="cuda", generator=g).bfloat16()
    b = torch.randn(K, N, device="cuda", generator=g).bfloat16()
    c = torch.randn(M, N, device="cuda", generator=g)
    ref = (c if accumulate else torch.zeros_like(c)) + 0.75 * (a.float().t() @ b.float())
    torch.ops.sxe.wgrad_gemm_variant_(a, b, c, 0.75, accumulate, variant)
    assert _rel(c, ref) < 1e-5


@pytest.mark.parametrize("K1,K2", [(128, 128), (256, 1024), (32, 96), (1024, 0)])
@pytest.mark.parametrize("accumulate", [True, False])
def test_wgrad_gemm_two_segments_vs_fp32_reference(K1, K2, accumulate):
    """wgrad_gemm2_: C (+)= alpha [A1; A2]^T [B1; B2] read from two K segments in place (the deferred
    expert weight gradients) == fp32 reference of the concatenated product; segments are slices of
    larger row-major buffers (equal leading dims)."""
    M, N = 512, 768
    g = torch.Generator(device="cuda").manual_seed(K1 + 7 * K2)
    big_a = torch.randn(K1 + K2 + 64, M, device="cuda", generator=g).bfloat16()
    big_b = torch.randn(K1 + K2 + 64, N, device="cuda", generator=g).bfloat16()
    a1, a2 = big_a[:K1], big_a[K1 + 64:]
    b1, b2 = big_b[:K1], big_b[K1 + 64:]
    c = torch.randn(M, N, device="cuda", generator=g)
    ref = (c if accumulate else torch.zeros_like(c)) + 0.5 * (torch.cat([a1, a2]).float().t() @ torch.cat([b1, b2]).float())
    torch.ops.sxe.wgrad_gemm2_(a1, b1, a2, b2, c, 0.5, accumulate)
    assert _rel(c, ref) < 1e-5


def test_grouped_mm_deferred_wgrad_two_segment_kernel_matches(monkeypatch):
    """moe/experts.py: a weight gradient deferred over two micro-steps goes through wgrad_gemm2_ at the
    boundary (no concatenation) and equals the fp32 sum of both micro-steps."""
    from shuffle_exchange_amd.moe import experts as E
    w = torch.nn.Parameter(torch.randn(1, 4096, 4096, device="cuda", dtype=torch.bfloat16) * 0.02)
    buf = torch.full((1, 4096, 4096), float("nan"), device="cuda")
    st = {"valid": False, "boundary": False, "done": 0, "two": 0}
    w._sxe_grad_target = lambda p: (buf, st["valid"])
    w._sxe_grad_done = lambda p: st.update(valid=True, done=st["done"] + 1)
    w._sxe_grad_defer = lambda p: not st["boundary"]
    real = E._wgrad2_ok

    def counted(*a):
        ok = real(*a)
        st["two"] += ok
        return ok
    monkeypatch.setattr(E, "_wgrad2_ok", counted)
    ref = torch.zeros(1, 4096, 4096, device="cuda")
    for k in range(2):
        st["boundary"] = k == 1
        x = torch.randn(1, 256, 4096, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        gy = torch.randn(1, 256, 4096, device="cuda", dtype=torch.bfloat16)
        ref += torch.einsum("eck,ecn->ekn", x.detach().float(), gy.float())
        E.grouped_mm(x, w).backward(gy)
    assert st["done"] == 1 and st["two"] == 1
    assert _rel(buf, ref) < 1e-5


def test_linear_weight_grad_uses_wgrad_kernel_and_matches():
    """ops/linear routes a (4096 x 4096)-class fp32-accumulated weight gradient through the HIP kernel;
    result == fp32 reference accumulated over two micro-steps."""
    from shuffle_exchange_amd.ops import linear as L
    w = torch.nn.Parameter(torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16) * 0.02)
    buf = torch.zeros(4096, 4096, device="cuda")
    state = {"n": 0, "done": 0}

    def tgt(p):
        state["n"] += 1
        return buf, state["n"] > 1

    w._sxe_grad_target = tgt
    w._sxe_grad_done = lambda p: state.__setitem__("done", state["done"] + 1)
    ref = torch.zeros(4096, 4096, device="cuda")
    for i in range(2):
        x = torch.randn(2, 1024, 4096, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        gy = torch.randn(2, 1024, 4096, device="cuda", dtype=torch.bfloat16)
        assert L._sxe_wgrad_ok(gy.reshape(-1, 4096), x.detach().reshape(-1, 4096), buf)
        y = L.linear(x, w)
        y.backward(gy)
        ref += gy.reshape(-1, 4096).float().t() @ x.detach().reshape(-1, 4096).float()
    assert state["done"] == 2 and w.grad is None
    assert _rel(buf, ref) < 1e-5


def test_lamb_kernels_vs_torch_reference():
    """optim.hip lamb_stage1_/lamb_stage2_ (per-segment trust ratios, bf16 copy) == fp32 torch LAMB."""
    from shuffle_exchange_amd.ops.optim import lamb_block_table, lamb_flat_
    torch.manual_seed(0)
    sizes = [1, 37, 8192, 8193, 100_000, 3]
    n = sum(sizes)
    p = torch.randn(n, device="cuda")
    g = torch.randn(n, device="cuda").bfloat16()
    m = torch.randn(n, device="cuda") * 0.01
    v = torch.rand(n, device="cuda") * 0.01
    lp = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    segs, off = [], 0
    for i, s in enumerate(sizes):
        segs.append((i, off, s))
        off += s
    ref_p, ref_m, ref_v = p.clone().cpu(), m.clone().cpu(), v.clone().cpu()
    coeffs = torch.empty(len(sizes), device="cuda")
    scale = torch.tensor([0.5], device="cuda")
    lamb_flat_(p, g, m, v, lp, lamb_block_table(segs, "cuda"), len(sizes), lr=1e-2, beta1=0.9, beta2=0.99, eps=1e-6,
               weight_decay=0.05, step=4, scale_t=scale, coeffs=coeffs)
    gf = g.float().cpu() * 0.5
    ref_m = 0.9 * ref_m + 0.1 * gf
    ref_v = 0.99 * ref_v + 0.01 * gf * gf
    u = (ref_m / (1 - 0.9 ** 4)) / ((ref_v / (1 - 0.99 ** 4)).sqrt() + 1e-6) + 0.05 * ref_p
    out = ref_p.clone()
    for i, s0, s in segs:
        wn, un = ref_p[s0:s0 + s].norm(), u[s0:s0 + s].norm()
        c = float((wn / un).clamp(0.01, 10.0)) if wn > 0 and un > 0 else 1.0
        assert abs(float(coeffs[i]) - c) < 1e-4 * max(1.0, c)
        out[s0:s0 + s] -= 1e-2 * c * u[s0:s0 + s]
    assert _rel(m.cpu(), ref_m) < 1e-6 and _rel(v.cpu(), ref_v) < 1e-6
    assert _rel(p.cpu(), out) < 1e-6
    assert torch.equal(lp, p.bfloat16())
