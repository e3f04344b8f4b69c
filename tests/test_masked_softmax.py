"""HIP masked softmax (csrc/kernels/softmax.hip) vs the fp32 PyTorch path of
ops.inference_ops.softmax: additive and boolean broadcast masks, ALiBi, causal, local window."""
import pytest
import torch

from shuffle_exchange_amd.ops import inference_ops


def _ref(s, **kw):
    return inference_ops.softmax(s.float().cpu(), **{k: (v.cpu() if torch.is_tensor(v) else v) for k, v in kw.items()})


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_masked_softmax_gpu(dtype):
    from shuffle_exchange_amd.ops import native
    native.require_hip()
    torch.manual_seed(0)
    B, H, Q, K = 2, 3, 5, 200
    s = (torch.randn(B, H, Q, K) * 3).to("cuda", dtype)
    pad = torch.rand(B, 1, 1, K, device="cuda") > 0.2
    add = torch.randn(B, 1, Q, K, device="cuda")
    alibi = torch.randn(1, H, 1, K, device="cuda")
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    cases = [dict(), dict(attn_mask=pad), dict(attn_mask=add, alibi=alibi), dict(triangular=True),
             dict(triangular=True, local_attention=True, window_size=7, layer_scale=0.5),
             dict(attn_mask=torch.zeros(B, 1, 1, K, dtype=torch.bool, device="cuda"))]
    for kw in cases:
        out = inference_ops.softmax(s, **kw)
        ref = _ref(s, **kw)
        ref = torch.nan_to_num(ref, nan=0.0)  # fully masked rows: the kernel outputs zeros
        assert out.dtype == dtype
        torch.testing.assert_close(out.float().cpu(), ref, rtol=tol, atol=tol)
