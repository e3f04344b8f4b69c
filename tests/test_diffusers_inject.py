"""Generic (diffusers-style) injection (module_inject/diffusers.py; reference generic_injection +
containers/unet.py / vae.py). diffusers is not installed: ``Attention`` below mirrors diffusers'
``Attention`` + ``AttnProcessor2_0`` forward (self / cross attention, 4-D VAE input, GroupNorm,
residual, rescale) and the fused modules must reproduce it. Parity vs diffusers itself: unpinned."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from shuffle_exchange_amd.module_inject.diffusers import FusedDiffusersAttention, generic_injection


class Attention(nn.Module):
    def __init__(self, query_dim, cross_attention_dim=None, heads=8, dim_head=64, bias=False, out_bias=True,
                 residual_connection=False, rescale_output_factor=1.0, norm_num_groups=None):
        super().__init__()
        inner = heads * dim_head
        kv_dim = cross_attention_dim or query_dim
        self.heads, self.scale = heads, dim_head ** -0.5
        self.residual_connection, self.rescale_output_factor = residual_connection, rescale_output_factor
        self.to_q = nn.Linear(query_dim, inner, bias=bias)
        self.to_k = nn.Linear(kv_dim, inner, bias=bias)
        self.to_v = nn.Linear(kv_dim, inner, bias=bias)
        self.to_out = nn.ModuleList([nn.Linear(inner, query_dim, bias=out_bias), nn.Dropout(0.0)])
        self.group_norm = nn.GroupNorm(norm_num_groups, query_dim, eps=1e-6) if norm_num_groups else None
        self.spatial_norm = self.norm_cross = None

    def forward(self, hidden_states, encoder_hidden_states=None, attention_mask=None):
        residual, nd = hidden_states, hidden_states.ndim
        if nd == 4:
            B, C, H, W = hidden_states.shape
            hidden_states = hidden_states.view(B, C, H * W).transpose(1, 2)
        if self.group_norm is not None:
            hidden_states = self.group_norm(hidden_states.transpose(1, 2)).transpose(1, 2)
        B = hidden_states.shape[0]
        ctx = hidden_states if encoder_hidden_states is None else encoder_hidden_states
        q, k, v = self.to_q(hidden_states), self.to_k(ctx), self.to_v(ctx)
        hd = q.shape[-1] // self.heads
        q, k, v = (t.view(B, -1, self.heads, hd).transpose(1, 2) for t in (q, k, v))
        o = F.scaled_dot_product_attention(q, k, v, attn_mask=attention_mask, scale=self.scale)
        o = self.to_out[1](self.to_out[0](o.transpose(1, 2).reshape(B, -1, self.heads * hd)))
        if nd == 4:
            o = o.transpose(-1, -2).reshape(B, C, H, W)
        if self.residual_connection:
            o = o + residual
        return o / self.rescale_output_factor


class BasicTransformerBlock(nn.Module):  # UNet cross-attention block: attn1 (self) + attn2 (cross)
    def __init__(self, dim, ctx_dim, heads, dim_head):
        super().__init__()
        self.norm1, self.norm2 = nn.LayerNorm(dim), nn.LayerNorm(dim)
        self.attn1 = Attention(dim, heads=heads, dim_head=dim_head)
        self.attn2 = Attention(dim, cross_attention_dim=ctx_dim, heads=heads, dim_head=dim_head)

    def forward(self, x, ctx):
        x = x + self.attn1(self.norm1(x))
        return x + self.attn2(self.norm2(x), encoder_hidden_states=ctx)


class VAEMidAttention(nn.Module):
    def __init__(self, ch):
        super().__init__()
        self.attention = Attention(ch, heads=1, dim_head=ch, bias=True, residual_connection=True,
                                   rescale_output_factor=1.0, norm_num_groups=8)

    def forward(self, x):
        return self.attention(x)


def _models(dev, dtype, dim_head):
    torch.manual_seed(0)
    unet = BasicTransformerBlock(dim=2 * dim_head, ctx_dim=96, heads=2, dim_head=dim_head).to(dev, dtype).eval()
    vae = VAEMidAttention(64).to(dev, dtype).eval()
    return unet, vae


def _check(dev, dtype, dim_head, tol):
    unet, vae = _models(dev, dtype, dim_head)
    x = torch.randn(2, 128, 2 * dim_head, device=dev, dtype=dtype)
    ctx = torch.randn(2, 77, 96, device=dev, dtype=dtype)
    img = torch.randn(2, 64, 8, 16, device=dev, dtype=dtype)
    with torch.no_grad():
        ref_u, ref_v = unet(x, ctx), vae(img)
        assert generic_injection(unet) == 2 and generic_injection(vae) == 1
        assert isinstance(unet.attn1, FusedDiffusersAttention) and isinstance(vae.attention, FusedDiffusersAttention)
        assert unet.attn1.self_only and not unet.attn2.self_only
        out_u, out_v = unet(x, ctx), vae(img)
        # a masked call is delegated to the original module and stays exact
        m = torch.zeros(2, 1, 128, 128, device=dev, dtype=dtype)
        torch.testing.assert_close(unet.attn1(x, attention_mask=m), unet.attn1.orig(x, attention_mask=m))
    for a, b in ((out_u, ref_u), (out_v, ref_v)):
        err = ((a.float() - b.float()).norm() / b.float().norm()).item()
        assert err < tol, err
    # the original modules hold views of the fused tensors, not copies
    assert unet.attn1.orig.to_k.weight.data_ptr() == unet.attn1.w_qkv[2 * dim_head:].data_ptr()
    assert unet.attn2.orig.to_v.weight.data_ptr() == unet.attn2.w_kv[2 * dim_head:].data_ptr()


def test_generic_injection_cpu():
    _check("cpu", torch.float32, 32, 1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("dim_head", [40, 64, 80])
def test_generic_injection_gpu_bf16(dim_head, monkeypatch):
    from shuffle_exchange_amd.module_inject import replace_module
    from shuffle_exchange_amd.ops import native
    native.require_hip()
    calls = []
    real = replace_module.attention
    monkeypatch.setattr(replace_module, "attention", lambda *a, **k: calls.append(1) or real(*a, **k))
    _check("cuda", torch.bfloat16, dim_head, 3e-2)
    assert len(calls) == 2, "UNet self-attention and the VAE attention must run the HIP flash kernel"


def test_init_inference_applies_generic_injection():
    import shuffle_exchange_amd as sxe
    unet, _ = _models("cpu", torch.float32, 32)
    eng = sxe.init_inference(unet, dtype=torch.float32, replace_with_kernel_inject=True)
    assert eng.injected_layers == 2 and isinstance(unet.attn2, FusedDiffusersAttention)
