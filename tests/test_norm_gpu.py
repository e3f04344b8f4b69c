"""RMSNorm / LayerNorm HIP kernels (csrc/kernels/norm.hip) in both forms -- the exact-width variant
(hidden a multiple of 512: no per-chunk bounds checks, every chunk's loads issued before the residual
stores) and the bounds-checked one (SXE_NORM_EXACT=0, or a ragged hidden size) -- against a plain
fp32 PyTorch reference of the same op, forward (with the fused residual add) and backward."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from shuffle_exchange_amd.ops import native
    native.require_hip()


def _ref_fwd(x, res, w, b, eps, ln):
    h = (x.float() + res.float()).bfloat16().float() if res is not None else x.float()
    if ln:
        mu = h.mean(-1, keepdim=True)
        y = (h - mu) * torch.rsqrt(((h - mu) ** 2).mean(-1, keepdim=True) + eps) * w.float() + b.float()
    else:
        y = h * torch.rsqrt((h * h).mean(-1, keepdim=True) + eps) * w.float()
    return y, h


@pytest.mark.parametrize("exact", ["1", "0"])
@pytest.mark.parametrize("H", [4096, 1024, 4104])
@pytest.mark.parametrize("ln", [False, True])
def test_norm_fwd_bwd_vs_fp32(exact, H, ln, monkeypatch):
    monkeypatch.setenv("SXE_NORM_EXACT", exact)
    torch.manual_seed(H)
    R, eps = 1000, 1e-5
    x = torch.randn(R, H, device="cuda", dtype=torch.bfloat16)
    res = torch.randn_like(x)
    w = (torch.rand(H, device="cuda") + 0.5).bfloat16()
    b = torch.randn(H, device="cuda").bfloat16() if ln else None
    y, rstd, mean, h = torch.ops.sxe.norm_fwd(x, res, w, b, eps, ln)
    ry, rh = _ref_fwd(x, res, w, b if ln else torch.zeros_like(w), eps, ln)
    torch.testing.assert_close(h.float(), rh, rtol=0, atol=0)
    torch.testing.assert_close(y.float(), ry, rtol=2e-2, atol=2e-2)
    # backward with a residual gradient added into dx
    dy = torch.randn_like(x)
    dres = torch.randn_like(x)
    dx, dw, db = torch.ops.sxe.norm_bwd(dy, h, rstd, mean if ln else None, w, dres, ln)
    hr = h.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    br = (b.float() if ln else torch.zeros(H, device="cuda")).requires_grad_(True)
    if ln:
        mu = hr.mean(-1, keepdim=True)
        out = (hr - mu) * torch.rsqrt(((hr - mu) ** 2).mean(-1, keepdim=True) + eps) * wr + br
    else:
        out = hr * torch.rsqrt((hr * hr).mean(-1, keepdim=True) + eps) * wr
    gx, gw, gb = torch.autograd.grad(out, (hr, wr, br), dy.float(), allow_unused=True)
    torch.testing.assert_close(dx.float(), gx + dres.float(), rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(dw, gw, rtol=1e-3, atol=1e-2)
    if ln:
        torch.testing.assert_close(db, gb, rtol=1e-3, atol=1e-2)
