"""Block-sparse attention (reference ops/sparse_attention): layout generators reproduce the reference
patterns; SparseSelfAttention == dense attention restricted to the layout; the gfx950 block-sparse
flash kernels (GPU) match the fp32 oracle in forward and backward."""
import pytest
import torch


def test_fixed_layout_pattern():
    from shuffle_exchange_amd.ops.sparse_attention import FixedSparsityConfig
    lay = FixedSparsityConfig(num_heads=2, block=16, num_local_blocks=4, num_global_blocks=1,
                              attention="bidirectional").make_layout(16 * 8)[0]
    # local 4x4 windows on the diagonal, global column = last block of each window (3, 7)
    exp = torch.zeros(8, 8, dtype=torch.int64)
    exp[0:4, 0:4] = 1
    exp[4:8, 4:8] = 1
    exp[:, 3] = 1
    exp[:, 7] = 1
    assert torch.equal(lay, exp)
    uni = FixedSparsityConfig(num_heads=1, block=16, num_local_blocks=4, attention="unidirectional").make_layout(128)[0]
    assert torch.equal(uni, torch.tril(uni))


def test_other_layouts_shapes_and_properties():
    from shuffle_exchange_amd.ops import sparse_attention as sa
    S = 16 * 16
    bb = sa.BigBirdSparsityConfig(4, block=16, num_random_blocks=2, num_sliding_window_blocks=3,
                                  num_global_blocks=1).make_layout(S)
    assert bb.shape == (4, 16, 16) and torch.equal(bb[0], bb[3])
    assert bb[0, 0].all() and bb[0, :, 0].all() and all(bb[0, i, i] for i in range(16))
    lf = sa.BSLongformerSparsityConfig(2, block=16, num_sliding_window_blocks=3, global_block_indices=[2],
                                       attention="unidirectional").make_layout(S)[0]
    assert torch.equal(lf, torch.tril(lf)) and lf[5, 2] == 1 and lf[5, 4] == 1 and lf[5, 3] == 0 and lf[5, 6] == 0
    loc = sa.LocalSlidingWindowSparsityConfig(1, block=16, num_sliding_window_blocks=5).make_layout(S)[0]
    assert loc[10, 8] == 1 and loc[10, 11] == 0 and loc[10, 7] == 0
    var = sa.VariableSparsityConfig(1, block=16, local_window_blocks=[2, 4], global_block_indices=[0],
                                    global_block_end_indices=[1]).make_layout(S)[0]
    assert var[0:2, 0:2].all() and var[2:6, 2:6].all() and var[:, 0].all() and var[6:10, 6:10].all()
    dense = sa.DenseSparsityConfig(2, block=16).make_layout(S)
    assert dense.all()


def test_sparse_self_attention_dense_layout_equals_attention():
    from shuffle_exchange_amd.ops.attention import reference_attention
    from shuffle_exchange_amd.ops.sparse_attention import DenseSparsityConfig, SparseSelfAttention
    torch.manual_seed(0)
    q, k, v = (torch.randn(2, 4, 64, 32) for _ in range(3))
    out = SparseSelfAttention(DenseSparsityConfig(4, block=16))(q, k, v)
    ref = reference_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), causal=False).transpose(1, 2)
    assert torch.allclose(out, ref, atol=1e-5)


from shuffle_exchange_amd.ops.sparse_attention import sparse_attention_reference as _REF  # noqa: E402


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,causal,hk,D", [
    ("fixed16", False, 4, 128), ("bigbird32", False, 4, 128), ("longformer64_uni", True, 4, 128),
    ("local128", True, 2, 128), ("fixed16", False, 1, 128), ("fixed16", False, 4, 64), ("bigbird32", True, 2, 64),
    ("longformer64_uni", True, 4, 96), ("local128", False, 2, 256)])
def test_block_sparse_flash_matches_reference(cfg, causal, hk, D, monkeypatch):
    """Every head dim runs the flash kernels (BERT's 64 included): the reference path must not run."""
    from shuffle_exchange_amd.ops import native
    from shuffle_exchange_amd.ops import sparse_attention as sa
    native.require_hip()
    torch.manual_seed(0)
    B, H, S = 2, 4, 512
    monkeypatch.setattr(sa, "sparse_attention_reference", None)
    ref_fn = _REF
    conf = {"fixed16": lambda: sa.FixedSparsityConfig(H, block=16, num_local_blocks=4, different_layout_per_head=True,
                                                      num_different_global_patterns=2),
            "bigbird32": lambda: sa.BigBirdSparsityConfig(H, block=32, num_random_blocks=1),
            "longformer64_uni": lambda: sa.BSLongformerSparsityConfig(H, block=64, attention="unidirectional"),
            "local128": lambda: sa.LocalSlidingWindowSparsityConfig(H, block=128, num_sliding_window_blocks=3)}[cfg]()
    layout = conf.make_layout(S)
    q = torch.randn(B, H, S, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, hk, S, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, hk, S, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    o = sa.block_sparse_attention(q, k, v, layout, conf.block, causal=causal)
    q2, k2, v2 = (t.detach().float().requires_grad_() for t in (q, k, v))
    o2 = ref_fn(q2, k2, v2, layout.cuda(), conf.block, D ** -0.5, causal)
    assert _rel(o, o2) < 1e-2
    g = torch.randn_like(o2)
    (o.float() * g).sum().backward()
    (o2 * g).sum().backward()
    for a, b in ((q.grad, q2.grad), (k.grad, k2.grad), (v.grad, v2.grad)):
        assert _rel(a, b) < 2e-2
