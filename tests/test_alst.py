"""ALST helpers: tiled MLP == plain MLP (values and grads), SP cross-entropy gather, HF Ulysses
attention adapter == single-rank attention (gloo, SP=2)."""
import torch

from .dist_utils import run_dist


def test_tiled_mlp_matches():
    from shuffle_exchange_amd.sequence import TiledMLP
    torch.manual_seed(0)
    mlp = torch.nn.Sequential(torch.nn.Linear(16, 64), torch.nn.SiLU(), torch.nn.Linear(64, 16))
    x = torch.randn(2, 40, 16, requires_grad=True)
    y = mlp(x)
    y.pow(2).sum().backward()
    ref = [x.grad.clone()] + [p.grad.clone() for p in mlp.parameters()]
    x.grad = None
    mlp.zero_grad()
    y2 = TiledMLP(mlp, num_shards=7)(x)
    assert torch.allclose(y, y2, atol=1e-6)
    y2.pow(2).sum().backward()
    got = [x.grad] + [p.grad for p in mlp.parameters()]
    for a, b in zip(ref, got):
        assert torch.allclose(a, b, atol=1e-5)


def _case_hf_attn(rank, world):
    import torch.nn.functional as F
    from shuffle_exchange_amd.parallel import groups
    from shuffle_exchange_amd.sequence.tiled import UlyssesSPAttentionHF, vocab_sequence_parallel_cross_entropy
    groups.initialize(sequence_parallel_size=world)
    g = groups.get_sequence_parallel_group()

    def core(module, q, k, v, mask, **kw):  # HF convention: in [B, H, S, D], out [B, S, H, D]
        if k.shape[1] != q.shape[1]:
            k = k.repeat_interleave(q.shape[1] // k.shape[1], 1)
            v = v.repeat_interleave(q.shape[1] // v.shape[1], 1)
        return F.scaled_dot_product_attention(q, k, v, is_causal=True).transpose(1, 2), None

    torch.manual_seed(0)
    B, H, Hk, S, D = 2, 4, 2, 16, 8
    q, k, v = torch.randn(B, H, S, D), torch.randn(B, Hk, S, D), torch.randn(B, Hk, S, D)
    full, _ = core(None, q, k, v, None)
    sl = slice(rank * S // world, (rank + 1) * S // world)
    fn = UlyssesSPAttentionHF(core, g, H, Hk, D)
    out, _ = fn(None, q[:, :, sl], k[:, :, sl], v[:, :, sl])
    logits = torch.randn(S, 3, 11)
    tgt = torch.randint(0, 11, (S, 3))
    loss = vocab_sequence_parallel_cross_entropy(logits[sl], tgt[sl], g)
    ref = F.cross_entropy(logits.reshape(-1, 11), tgt.reshape(-1), reduction="none").view(S, 3)
    return {"ok": bool(torch.allclose(out, full[:, sl], atol=1e-5)), "ce": bool(torch.allclose(loss, ref, atol=1e-5))}


def test_hf_ulysses_adapter_and_sp_ce():
    for r in run_dist(_case_hf_attn, 2):
        assert r["ok"] and r["ce"]
