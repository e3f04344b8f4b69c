"""FPDT (reference deepspeed/sequence/fpdt_layer.py): chunked, load-balanced sequence-parallel
attention must equal full causal attention of the global sequence -- outputs and input gradients --
on one rank (chunking only) and on 2 gloo ranks (chunking + Ulysses all-to-all); the chunked FFN and
logits-loss functions must equal their eager counterparts."""
import torch

from .dist_utils import run_dist


def _global_problem(B=2, S=64, nq=4, nkv=2, D=16, seed=0):
    g = torch.Generator().manual_seed(seed)
    qkv = torch.randn(B, S, nq + 2 * nkv, D, generator=g)
    w = torch.randn(B, S, nq, D, generator=g)
    return qkv, w


def _reference(qkv, w, nq, nkv, rope):
    from shuffle_exchange_amd.ops.attention import reference_attention
    from shuffle_exchange_amd.ops.rope import apply_rope_qkv_
    x = qkv.clone().requires_grad_(True)
    r = apply_rope_qkv_(x, rope, nq + nkv)
    o = reference_attention(r[:, :, :nq], r[:, :, nq:nq + nkv], r[:, :, nq + nkv:], True)
    (o * w).sum().backward()
    return o.detach(), x.grad


def _rope(D, S):
    from shuffle_exchange_amd.ops.rope import RopeCache
    return RopeCache(D, S, 10000.0)


def test_update_out_and_lse_matches_joint_softmax():
    from shuffle_exchange_amd.ops.attention import reference_attention
    from shuffle_exchange_amd.sequence.fpdt_layer import update_out_and_lse
    torch.manual_seed(0)
    q, k, v = torch.randn(1, 8, 2, 16), torch.randn(1, 16, 2, 16), torch.randn(1, 16, 2, 16)
    full, full_lse = reference_attention(q, k, v, False, return_lse=True)
    out = lse = None
    for j in range(2):
        bo, bl = reference_attention(q, k[:, 8 * j:8 * j + 8], v[:, 8 * j:8 * j + 8], False, return_lse=True)
        out, lse = update_out_and_lse(out, lse, bo, bl)
    assert torch.allclose(out, full, atol=1e-5) and torch.allclose(lse, full_lse, atol=1e-5)


def test_fpdt_single_rank_chunks_match_full_attention():
    from shuffle_exchange_amd.sequence.fpdt_layer import fpdt_attention
    nq, nkv, D, S = 4, 2, 16, 64
    qkv, w = _global_problem(S=S, nq=nq, nkv=nkv, D=D)
    rope = _rope(D, S)
    ref_o, ref_g = _reference(qkv, w, nq, nkv, rope)
    x = qkv.clone().requires_grad_(True)
    o = fpdt_attention(x, nq, nkv, rope, None, num_chunks=4)
    (o * w).sum().backward()
    assert torch.allclose(o, ref_o, atol=1e-4), (o - ref_o).abs().max()
    assert torch.allclose(x.grad, ref_g, atol=1e-4), (x.grad - ref_g).abs().max()


def _case_fpdt_sp(rank, world, chunk_size):
    import shuffle_exchange_amd.comm as dist
    from shuffle_exchange_amd.sequence.fpdt_layer import FPDT_InputConstruct, fpdt_attention
    nq, nkv, D, S = 4, 2, 16, 64
    qkv, w = _global_problem(S=S, nq=nq, nkv=nkv, D=D)
    rope = _rope(D, S)
    ref_o, ref_g = _reference(qkv, w, nq, nkv, rope)
    group = dist.new_group(list(range(world)))
    ic = FPDT_InputConstruct(torch.zeros(2, S, dtype=torch.long), None, None, None, None, chunk_size, world, rank)
    idx = ic.indices()
    x = qkv[:, idx].clone().requires_grad_(True)
    o = fpdt_attention(x, nq, nkv, rope, group, num_chunks=ic.num_chunk_per_gpu)
    (o * w[:, idx]).sum().backward()
    return {"o": (o.detach() - ref_o[:, idx]).abs().max().item(),
            "g": (x.grad - ref_g[:, idx]).abs().max().item(), "idx": idx.tolist()}


def test_fpdt_sequence_parallel_matches_full_attention():
    res = run_dist(_case_fpdt_sp, 2, 16)
    for r in res:
        assert r["o"] < 1e-4 and r["g"] < 1e-4, r
    # load-balanced layout (reference fpdt_layer.py:92-123): S/chunk_size = 4 chunks per rank of
    # 8 tokens; rank r holds global 8-token chunks r, r+2, r+4, r+6
    assert res[0]["idx"] == [t for c in (0, 2, 4, 6) for t in range(8 * c, 8 * c + 8)]
    assert res[1]["idx"] == [t for c in (1, 3, 5, 7) for t in range(8 * c, 8 * c + 8)]


def test_fpdt_ffn_and_logits_loss_match_eager():
    from shuffle_exchange_amd.sequence.fpdt_layer import FPDT_FFN, FPDT_LogitsLoss, _gelu
    torch.manual_seed(0)
    x = torch.randn(32, 2, 8, requires_grad=True)
    w1, b1 = torch.randn(24, 8, requires_grad=True), torch.randn(24, requires_grad=True)
    w2, b2 = torch.randn(8, 24, requires_grad=True), torch.randn(8, requires_grad=True)
    out, _ = FPDT_FFN.apply(x, w1, b1, w2, b2, True, 8)
    g = torch.randn_like(out)
    grads = torch.autograd.grad(out, (x, w1, b1, w2, b2), g)
    ref = torch.matmul(_gelu(torch.matmul(x, w1.t()) + b1), w2.t()) + b2
    rgrads = torch.autograd.grad(ref, (x, w1, b1, w2, b2), g)
    assert torch.allclose(out, ref, atol=1e-4)
    for a, b in zip(grads, rgrads):
        assert torch.allclose(a, b, atol=1e-3, rtol=1e-4)

    h = torch.randn(2, 16, 8, requires_grad=True)
    wl = torch.randn(40, 8, requires_grad=True)
    lab = torch.randint(0, 40, (2, 16))
    loss = FPDT_LogitsLoss.apply(h, lab, wl, None, 4)
    gl = torch.randn_like(loss)
    gh, gw = torch.autograd.grad(loss, (h, wl), gl)
    rl = torch.nn.functional.cross_entropy(torch.matmul(h, wl.t()).reshape(-1, 40), lab.reshape(-1),
                                           reduction="none").view(2, 16)
    rh, rw = torch.autograd.grad(rl, (h, wl), gl)
    assert torch.allclose(loss, rl, atol=1e-4)
    assert torch.allclose(gh, rh, atol=1e-4) and torch.allclose(gw, rw, atol=1e-4)


def _case_fpdt_llama_train(rank, world):
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    from shuffle_exchange_amd.parallel import groups
    from shuffle_exchange_amd.sequence.fpdt_layer import FPDT_InputConstruct
    torch.manual_seed(0)
    cfg = llama_config("llama-tiny", sequence_parallel=True, fpdt_chunk_size=8)
    model = LlamaForCausalLM(cfg)
    ds = {"train_micro_batch_size_per_gpu": 2, "sequence_parallel_size": world,
          "zero_optimization": {"stage": 1}, "optimizer": {"type": "SGD", "params": {"lr": 0.1}}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    g = torch.Generator().manual_seed(11)
    losses = []
    for _ in range(2):
        ids = torch.randint(0, cfg.vocab_size, (2, 32), generator=g)
        labels = torch.cat([ids[:, 1:], torch.full_like(ids[:, :1], -100)], dim=1)  # shift globally first
        ic = FPDT_InputConstruct(ids, labels, None, None, None, 8, world, groups.get_sequence_parallel_rank())
        toks, labs, _, _, _ = ic.generate()
        loss = eng(toks, labels=labs, shift_labels=False)
        from shuffle_exchange_amd import comm
        tot = loss.detach().clone()
        comm.all_reduce(tot, group=groups.get_sequence_parallel_group())
        eng.backward(loss)
        eng.step()
        losses.append(float(tot))
    from ._dist_cases import full_params
    return {"losses": losses, "params": full_params(eng)}


def test_fpdt_llama_sp_training_matches_full_sequence():
    """Llama with FPDT attention on 2 SP ranks (load-balanced chunks) trains exactly like the
    single-process model on full sequences."""
    import pytest
    from .test_sequence_parallel import _reference_full_seq
    res = run_dist(_case_fpdt_llama_train, 2)
    ref = _reference_full_seq()
    for r in res:
        for a, b in zip(r["losses"], ref["losses"]):
            assert a == pytest.approx(b, rel=1e-5)
        for k, v in ref["params"].items():
            assert torch.allclose(r["params"][k], v, atol=2e-5), k
