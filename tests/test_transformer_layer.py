"""DeepSpeedTransformerLayer (ops/transformer.py) against transformers' BertLayer (Post-LN, the
reference's unit-test model) and a hand-written Pre-LN layer, forward and backward, fp32 on CPU."""
import pytest
import torch

transformers = pytest.importorskip("transformers")


def _bert(H=64, heads=4, I=256):
    cfg = transformers.BertConfig(hidden_size=H, num_attention_heads=heads, intermediate_size=I,
                                  hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0, hidden_act="gelu",
                                  layer_norm_eps=1e-12)
    cfg._attn_implementation = "eager"
    torch.manual_seed(0)
    return transformers.models.bert.modeling_bert.BertLayer(cfg).eval(), cfg


def _out(r):
    return r[0] if isinstance(r, tuple) else r


def _ds_from_bert(bl, cfg, pre_ln=False, **kw):
    from shuffle_exchange_amd.ops.transformer import DeepSpeedTransformerConfig, DeepSpeedTransformerLayer
    c = DeepSpeedTransformerConfig(batch_size=2, hidden_size=cfg.hidden_size, intermediate_size=cfg.intermediate_size,
                                   heads=cfg.num_attention_heads, attn_dropout_ratio=0.0, hidden_dropout_ratio=0.0,
                                   num_hidden_layers=2, initializer_range=0.02, layer_norm_eps=1e-12,
                                   pre_layer_norm=pre_ln, **kw)
    a, o, i, out = bl.attention.self, bl.attention.output, bl.intermediate, bl.output
    ws = [a.query.weight, a.key.weight, a.value.weight, o.dense.weight, o.LayerNorm.weight, i.dense.weight,
          out.dense.weight, out.LayerNorm.weight]
    bs = [a.query.bias, a.key.bias, a.value.bias, o.dense.bias, o.LayerNorm.bias, i.dense.bias, out.dense.bias,
          out.LayerNorm.bias]
    ws = [torch.nn.Parameter(w.detach().clone()) for w in ws]
    bs = [torch.nn.Parameter(b.detach().clone()) for b in bs]
    layer = DeepSpeedTransformerLayer(c, ws, bs).eval()
    layer.attn_qkvb = torch.nn.Parameter(torch.cat([bs[0].data, bs[1].data, bs[2].data]))
    return layer


@pytest.mark.parametrize("with_mask", [False, True])
@pytest.mark.parametrize("ckpt", [False, True])
def test_post_ln_matches_hf_bert_layer(with_mask, ckpt):
    bl, cfg = _bert()
    ds = _ds_from_bert(bl, cfg, gelu_checkpoint=ckpt, attn_dropout_checkpoint=ckpt).train()
    x = torch.randn(2, 16, cfg.hidden_size, requires_grad=True)
    mask = None
    if with_mask:
        keep = torch.ones(2, 16)
        keep[1, 11:] = 0
        mask = (1.0 - keep[:, None, None, :]) * torch.finfo(torch.float32).min
    ref = _out(bl(x, attention_mask=mask))
    out = ds(x, mask)
    torch.testing.assert_close(out, ref, atol=1e-5, rtol=1e-5)
    g = torch.randn_like(out)
    gx_ref, = torch.autograd.grad(ref, x, g)
    gx, = torch.autograd.grad(out, x, g)
    torch.testing.assert_close(gx, gx_ref, atol=1e-5, rtol=1e-4)
    ds.zero_grad()
    out = ds(x, mask)
    out.backward(g)
    ref2 = _out(bl(x, attention_mask=mask))
    ref2.backward(g)
    torch.testing.assert_close(ds.inter_w.grad, bl.intermediate.dense.weight.grad, atol=1e-5, rtol=1e-4)
    gq = ds.attn_qkvw.grad[:cfg.hidden_size]
    torch.testing.assert_close(gq, bl.attention.self.query.weight.grad, atol=1e-5, rtol=1e-4)


def test_pre_ln_formula():
    bl, cfg = _bert()
    ds = _ds_from_bert(bl, cfg, pre_ln=True)
    x = torch.randn(2, 16, cfg.hidden_size)
    F = torch.nn.functional
    H, nh = cfg.hidden_size, cfg.num_attention_heads
    a = F.layer_norm(x, (H,), ds.attn_nw, ds.attn_nb, 1e-12)
    qkv = (a @ ds.attn_qkvw.t() + ds.attn_qkvb).view(2, 16, 3, nh, H // nh)
    q, k, v = (qkv[:, :, i].transpose(1, 2) for i in range(3))
    ctx = torch.softmax(q @ k.transpose(-1, -2) / (H // nh) ** 0.5, -1) @ v
    h = x + ctx.transpose(1, 2).reshape(2, 16, H) @ ds.attn_ow.t() + ds.attn_ob
    m = F.layer_norm(h, (H,), ds.norm_w, ds.norm_b, 1e-12)
    ref = h + F.gelu(m @ ds.inter_w.t() + ds.inter_b) @ ds.output_w.t() + ds.output_b
    torch.testing.assert_close(ds(x), ref, atol=1e-5, rtol=1e-5)


def test_default_init_and_tuple_return():
    from shuffle_exchange_amd.ops.transformer import DeepSpeedTransformerConfig, DeepSpeedTransformerLayer
    c = DeepSpeedTransformerConfig(batch_size=2, hidden_size=32, heads=2, attn_dropout_ratio=0.1,
                                   hidden_dropout_ratio=0.1, num_hidden_layers=4, initializer_range=0.02,
                                   return_tuple=True)
    layer = DeepSpeedTransformerLayer(c)
    assert layer.inter_w.shape == (128, 32) and torch.all(layer.norm_w == 1)
    out = layer(torch.randn(2, 8, 32), torch.ones(2, 8))
    assert isinstance(out, tuple) and out[0].shape == (2, 8, 32)
