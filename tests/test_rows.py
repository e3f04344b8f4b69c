"""Row gather / scatter ops (csrc/kernels/rows.hip): ragged embedding with a vocab-shard offset,
last-token gather with the fused residual add, random-LTD token gather / scatter with autograd.
CPU cases check the fallback against torch indexing; GPU cases check the HIP kernels against the
same fp32 PyTorch reference and assert the native op ran."""
import pytest
import torch

from shuffle_exchange_amd.ops import rows


def _ref_gather(src, idx, offset=0, add=None):
    s = idx.long() - offset
    ok = (s >= 0) & (s < src.shape[0])
    out = torch.zeros(idx.numel(), src.shape[1], dtype=torch.float32, device=src.device)
    out[ok] = src.float()[s[ok]] + (add.float()[s[ok]] if add is not None else 0)
    return out


def _check(device, dtype):
    g = torch.Generator().manual_seed(0)
    src = torch.randn(50, 136, generator=g).to(device, dtype)
    add = torch.randn(50, 136, generator=g).to(device, dtype)
    idx = torch.randint(-5, 60, (77,), generator=g).to(device)
    for ix in (idx, idx.int()):
        torch.testing.assert_close(rows.gather_rows(src, ix, 0).float(), _ref_gather(src, ix), rtol=0, atol=0)
        torch.testing.assert_close(rows.gather_rows(src, ix, 10).float(), _ref_gather(src, ix, 10), rtol=0, atol=0)
        tol = 0 if dtype == torch.float32 else 1e-2
        torch.testing.assert_close(rows.gather_last(src, ix.clamp(0, 49), add).float(),
                                   _ref_gather(src, ix.clamp(0, 49), 0, add), rtol=tol, atol=tol)
    dst = torch.zeros(40, 136, device=device, dtype=dtype)
    perm = torch.randperm(40, generator=g)[:13].to(device)
    part = torch.randn(13, 136, generator=g).to(device, dtype)
    rows.scatter_rows_(dst, perm, part)
    ref = torch.zeros(40, 136, device=device, dtype=dtype)
    ref[perm] = part
    assert torch.equal(dst, ref)


def _check_tokens(device, dtype):
    torch.manual_seed(1)
    B, S, H, k = 3, 20, 64, 7
    x = torch.randn(B, S, H, device=device, dtype=dtype, requires_grad=True)
    idx = torch.sort(torch.stack([torch.randperm(S)[:k] for _ in range(B)]), -1).values.to(device)
    part = rows.gather_tokens(x, idx)
    ref = torch.gather(x, 1, idx.unsqueeze(-1).expand(-1, -1, H))
    assert torch.equal(part, ref)
    y = part * 2 + 1
    full = rows.scatter_tokens(x, y, idx)
    ref_full = x.scatter(1, idx.unsqueeze(-1).expand(-1, -1, H), torch.gather(x, 1, idx.unsqueeze(-1).expand(-1, -1, H)) * 2 + 1)
    assert torch.equal(full, ref_full)
    w = torch.randn_like(full)
    (g1,) = torch.autograd.grad((full * w).sum(), x)
    x2 = x.detach().clone().requires_grad_(True)
    r2 = x2.scatter(1, idx.unsqueeze(-1).expand(-1, -1, H), torch.gather(x2, 1, idx.unsqueeze(-1).expand(-1, -1, H)) * 2 + 1)
    (g2,) = torch.autograd.grad((r2 * w).sum(), x2)
    torch.testing.assert_close(g1.float(), g2.float(), rtol=0, atol=0)


def test_rows_cpu():
    _check("cpu", torch.float32)
    _check_tokens("cpu", torch.float32)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32, torch.float16])
def test_rows_gpu(dtype):
    from shuffle_exchange_amd.ops import native
    native.require_hip()
    _check("cuda", dtype)
    _check_tokens("cuda", dtype)
