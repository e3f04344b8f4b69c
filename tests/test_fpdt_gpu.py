"""FPDT on the gfx950 flash kernels: chunk-pair forward with LSE merge and the chunk-pair backward
fed with the merged output/LSE, with and without host offload of the saved chunks, against the
fp32 full-attention oracle (single rank: chunking only)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("offload", [False, True])
def test_fpdt_flash_chunks_match_full_attention(offload):
    from shuffle_exchange_amd.ops import native
    from shuffle_exchange_amd.ops.attention import reference_attention
    from shuffle_exchange_amd.ops.rope import RopeCache, apply_rope_qkv_
    from shuffle_exchange_amd.sequence.fpdt_layer import fpdt_attention
    native.require_hip()
    torch.manual_seed(0)
    B, S, nq, nkv, D = 1, 1024, 8, 2, 128
    rope = RopeCache(D, S, 500000.0, device="cuda")
    qkv = torch.randn(B, S, nq + 2 * nkv, D, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(B, S, nq, D, device="cuda", dtype=torch.float32)
    x = qkv.clone().requires_grad_(True)
    o = fpdt_attention(x, nq, nkv, rope, None, num_chunks=4, offload=offload)
    (o.float() * w).sum().backward()

    xr = qkv.detach().float().cpu().requires_grad_(True)
    rope_c = RopeCache(D, S, 500000.0)
    r = apply_rope_qkv_(xr, rope_c, nq + nkv)
    ref = reference_attention(r[:, :, :nq], r[:, :, nq:nq + nkv], r[:, :, nq + nkv:], True)
    (ref * w.cpu()).sum().backward()
    assert _rel(o.cpu(), ref) < 1e-2
    assert _rel(x.grad.cpu(), xr.grad) < 2e-2
