"""Standalone block-sparse MatMul (sdd / dsd / dds, with transposes) and Softmax (scale, rpe,
key-padding and attention masks) against dense fp32 PyTorch on the same layout (reference
ops/sparse_attention/matmul.py:628, softmax.py:224, bert_sparse_self_attention.py:10)."""
import pytest
import torch

from shuffle_exchange_amd.ops.sparse_ops import MatMul, Softmax, block_sparse_to_dense, dense_to_block_sparse

BLK, H, M = 16, 3, 4
S = BLK * M


def _layout(seed=0):
    g = torch.Generator().manual_seed(seed)
    lay = (torch.rand(H, M, M, generator=g) < 0.5).long()
    lay[:, torch.arange(M), torch.arange(M)] = 1  # every row has a block
    return lay


def _mask(lay):
    return lay.repeat_interleave(BLK, 1).repeat_interleave(BLK, 2).bool()


@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True), (True, True)])
def test_sdd(ta, tb):
    torch.manual_seed(0)
    lay = _layout()
    a = torch.randn(2, H, S, 40, dtype=torch.float64)
    b = torch.randn(2, H, 40, S, dtype=torch.float64)
    A = a.transpose(-1, -2).contiguous() if ta else a
    Bm = b.transpose(-1, -2).contiguous() if tb else b
    c = MatMul(lay, BLK, "sdd", trans_a=ta, trans_b=tb)(A, Bm)
    ref = dense_to_block_sparse(a @ b, lay, BLK)
    torch.testing.assert_close(c, ref)


@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True)])
def test_dsd_and_dds(ta, tb):
    torch.manual_seed(1)
    lay = _layout(1)
    sp_dense = torch.randn(2, H, S, S, dtype=torch.float64) * _mask(lay)
    sp = dense_to_block_sparse(sp_dense, lay, BLK)
    d = torch.randn(2, H, S, 24, dtype=torch.float64)
    D = d.transpose(-1, -2).contiguous() if tb else d
    A = dense_to_block_sparse(sp_dense.transpose(-1, -2), lay.transpose(1, 2), BLK) if ta else sp
    lay_a = lay.transpose(1, 2).contiguous() if ta else lay
    out = MatMul(lay_a, BLK, "dsd", trans_a=ta, trans_b=tb)(A, D)
    torch.testing.assert_close(out, sp_dense @ d)
    # dds: dense [B, H, Md, S] x sparse
    e = torch.randn(2, H, 24, S, dtype=torch.float64)
    E = e.transpose(-1, -2).contiguous() if ta else e
    Bs = dense_to_block_sparse(sp_dense.transpose(-1, -2), lay.transpose(1, 2), BLK) if tb else sp
    lay_b = lay.transpose(1, 2).contiguous() if tb else lay
    out2 = MatMul(lay_b, BLK, "dds", trans_a=ta, trans_b=tb)(E, Bs)
    torch.testing.assert_close(out2, e @ sp_dense)


def test_sdd_backward_matches_dense():
    torch.manual_seed(2)
    lay = _layout(2)
    a = torch.randn(1, H, S, 32, dtype=torch.float64, requires_grad=True)
    b = torch.randn(1, H, 32, S, dtype=torch.float64, requires_grad=True)
    g = torch.randn(1, int(lay.sum()), BLK, BLK, dtype=torch.float64)
    (MatMul(lay, BLK, "sdd")(a, b) * g).sum().backward()
    ga, gb = a.grad.clone(), b.grad.clone()
    a.grad = b.grad = None
    ((a @ b) * block_sparse_to_dense(g, lay, BLK)).sum().backward()
    torch.testing.assert_close(ga, a.grad)
    torch.testing.assert_close(gb, b.grad)


@pytest.mark.parametrize("mode", ["add", "mul"])
def test_softmax_with_masks(mode):
    torch.manual_seed(3)
    lay = _layout(3)
    x = torch.randn(2, H, S, S, dtype=torch.float64)
    rpe = torch.randn(H, S, S, dtype=torch.float64)
    kpm = torch.where(torch.rand(2, S) < 0.2, -1e4, 0.0).double() if mode == "add" else (torch.rand(2, S) > 0.2).double()
    am = torch.randn(S, S, dtype=torch.float64) if mode == "add" else (torch.rand(S, S) > 0.1).double()
    xs = dense_to_block_sparse(x, lay, BLK)
    y = Softmax(lay, BLK)(xs, scale=0.5, rpe=rpe, key_padding_mask=kpm, attn_mask=am,
                          key_padding_mask_mode=mode, attn_mask_mode=mode)
    s = x * 0.5 + rpe
    s = s + am if mode == "add" else s * am
    s = s + kpm.view(2, 1, 1, S) if mode == "add" else s * kpm.view(2, 1, 1, S)
    s = s.masked_fill(~_mask(lay), float("-inf"))
    ref = dense_to_block_sparse(torch.softmax(s, -1), lay, BLK)
    torch.testing.assert_close(y, ref)


def test_bert_sparse_self_attention_matches_dense_on_a_dense_layout():
    from types import SimpleNamespace

    from shuffle_exchange_amd.ops.sparse_attention import BertSparseSelfAttention, DenseSparsityConfig
    torch.manual_seed(4)
    cfg = SimpleNamespace(hidden_size=64, num_attention_heads=4)
    m = BertSparseSelfAttention(cfg, DenseSparsityConfig(num_heads=4, block=16))
    x = torch.randn(2, 32, 64)
    mask = torch.zeros(2, 32)
    out = m(x, mask)
    q, k, v = (m.transpose_for_scores(f(x)) for f in (m.query, m.key, m.value))
    ref = torch.softmax(q @ k.transpose(-1, -2) / 4.0, -1) @ v
    torch.testing.assert_close(out, ref.permute(0, 2, 1, 3).reshape(2, 32, 64), atol=1e-5, rtol=1e-4)
