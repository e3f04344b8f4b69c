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


# ------------------------------------------------------------------ HF model end to end (SP = 2)
def _hf_tiny(seed):
    from transformers import LlamaConfig, LlamaForCausalLM
    torch.manual_seed(seed)
    c = LlamaConfig(vocab_size=128, hidden_size=64, intermediate_size=128, num_hidden_layers=2,
                    num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=64)
    c._attn_implementation = "sdpa"
    return LlamaForCausalLM(c), c


def _hf_batches():
    g = torch.Generator().manual_seed(3)
    out = []
    for _ in range(2):  # one data-parallel batch per SP rank (the helper runs both)
        ids = torch.randint(0, 128, (2, 16), generator=g)
        lab = ids.clone()
        lab[0, :3] = -100
        out.append({"input_ids": ids, "labels": lab, "position_ids": torch.arange(16).expand(2, 16).clone()})
    return out


def _case_fwd_loss_bwd(rank, world, debug_skip):
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.parallel import groups
    from shuffle_exchange_amd.sequence.tiled import UlyssesSPFwdLossBwdWithLogits, register_with_transformers
    groups.initialize(sequence_parallel_size=world)
    model, cfg = _hf_tiny(0)
    fn = register_with_transformers(cfg, core_attn_implementation="sdpa", sp_group=groups.get_sequence_parallel_group())
    fn.skip_all_but_last_attention_debug_mode = debug_skip
    seen_pos = []
    core = fn.attn_fn

    def spy(module, q, k, v, mask, *a, **kw):
        seen_pos.append(tuple(kw["position_ids"].shape) if kw.get("position_ids") is not None else None)
        return core(module, q, k, v, mask, *a, **kw)
    fn.attn_fn = spy
    model.config._attn_implementation = "ulysses"
    ds = {"train_micro_batch_size_per_gpu": 2, "sequence_parallel_size": world,
          "zero_optimization": {"stage": 1}, "optimizer": {"type": "SGD", "params": {"lr": 0.5}}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    step = UlyssesSPFwdLossBwdWithLogits(eng, model, torch.device("cpu"))
    loss = step.sp_fwd_loss_bwd(dict(_hf_batches()[rank]))
    eng.step()
    return {"loss": loss, "params": {n: p.detach().clone() for n, p in model.named_parameters()},
            "pos": seen_pos}


def test_ulysses_fwd_loss_bwd_with_logits_matches_single_process():
    """UlyssesSPFwdLossBwdWithLogits on 2 SP ranks (HF Llama, GQA, core attention behind the Ulysses
    adapter with position_ids all-gathered) == one process running both batches unsharded."""
    res = run_dist(_case_fwd_loss_bwd, 2, False)
    model, _ = _hf_tiny(0)
    opt = torch.optim.SGD(model.parameters(), lr=0.5)
    losses = []
    for b in _hf_batches():
        out = model(input_ids=b["input_ids"], labels=b["labels"])
        out.loss.backward()
        losses.append(float(out.loss))
    opt.step()
    for r in res:
        assert abs(r["loss"] - sum(losses) / 2) < 1e-4, (r["loss"], losses)
        assert all(p == (2, 16) for p in r["pos"]), r["pos"]  # the 8-token shards gathered to 16
        for n, p in model.named_parameters():
            torch.testing.assert_close(r["params"][n], p.detach(), atol=2e-5, rtol=1e-4)


def test_skip_all_but_last_attention_debug_mode():
    res = run_dist(_case_fwd_loss_bwd, 2, True)
    # 2 layers x 2 sub-steps forward: the core runs only for every 2nd layer call
    for r in res:
        assert len(r["pos"]) == 2, r["pos"]
