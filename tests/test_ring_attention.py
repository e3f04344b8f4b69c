"""Ring attention (sequence/ring_attention.py) on gloo: each rank's chunk of the output and of the
q/k/v gradients equals full attention over the whole sequence (causal and not, GQA, p = 2 and 4),
and a Llama training step with ring context parallelism equals the single-process step."""
import pytest
import torch

from .dist_utils import run_dist


def _full(q, k, v, causal):
    G = q.shape[2] // k.shape[2]
    qt, kt, vt = (t.transpose(1, 2) for t in (q, k.repeat_interleave(G, 2), v.repeat_interleave(G, 2)))
    return torch.nn.functional.scaled_dot_product_attention(qt, kt, vt, is_causal=causal).transpose(1, 2)


def _case_ring(rank, world, causal, layout):
    from shuffle_exchange_amd.parallel import groups
    from shuffle_exchange_amd.sequence.ring_attention import ring_attention, zigzag_indices
    groups.initialize(sequence_parallel_size=world)
    g = groups.get_sequence_parallel_group()
    torch.manual_seed(0)
    B, S, H, Hk, D = 2, 6 * world, 4, 2, 8
    q, k, v = torch.randn(B, S, H, D), torch.randn(B, S, Hk, D), torch.randn(B, S, Hk, D)
    dy = torch.randn(B, S, H, D)
    # reference: full attention on the whole sequence
    qr, kr, vr = (t.clone().requires_grad_() for t in (q, k, v))
    ref = _full(qr, kr, vr, causal)
    ref.backward(dy)
    sl = zigzag_indices(S, rank, world) if layout == "zigzag" else torch.arange(rank * 6, (rank + 1) * 6)
    ql, kl, vl = (t[:, sl].clone().requires_grad_() for t in (q, k, v))
    out = ring_attention(ql, kl, vl, g, causal=causal, layout=layout)
    out.backward(dy[:, sl])
    err = lambda a, b: float((a - b).abs().max())  # noqa: E731
    return {"o": err(out, ref[:, sl]), "dq": err(ql.grad, qr.grad[:, sl]), "dk": err(kl.grad, kr.grad[:, sl]),
            "dv": err(vl.grad, vr.grad[:, sl])}


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("layout", ["contiguous", "zigzag"])
def test_ring_attention_equals_full(world, causal, layout):
    for r in run_dist(_case_ring, world, causal, layout):
        assert max(r.values()) < 1e-5, r


def _case_ring_llama(rank, world, mode):
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd import comm
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    from shuffle_exchange_amd.parallel import groups
    from shuffle_exchange_amd.sequence.data import shard_batch_for_sp
    from shuffle_exchange_amd.sequence.ring_attention import zigzag_shard
    shard = zigzag_shard if mode == "ring_zigzag" else shard_batch_for_sp
    torch.manual_seed(0)
    cfg = llama_config("llama-tiny", sequence_parallel=True, sp_mode=mode)
    model = LlamaForCausalLM(cfg)
    ds = {"train_micro_batch_size_per_gpu": 2, "sequence_parallel_size": world,
          "zero_optimization": {"stage": 1}, "optimizer": {"type": "SGD", "params": {"lr": 0.1}}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    g = torch.Generator().manual_seed(11)
    losses = []
    for _ in range(2):
        ids = torch.randint(0, cfg.vocab_size, (2, 32), generator=g)
        b = shard(ids, groups.get_sequence_parallel_rank(), world)
        loss = eng(b["input_ids"], labels=b["labels"], position_ids=b["position_ids"], shift_labels=False)
        tot = loss.detach().clone()
        comm.all_reduce(tot, group=groups.get_sequence_parallel_group())
        eng.backward(loss)
        eng.step()
        losses.append(float(tot))
    return {"losses": losses}


@pytest.mark.parametrize("mode", ["ring", "ring_zigzag"])
def test_ring_context_parallel_llama_step(mode):
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    torch.manual_seed(0)
    model = LlamaForCausalLM(llama_config("llama-tiny"))
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    g = torch.Generator().manual_seed(11)
    ref = []
    for _ in range(2):
        ids = torch.randint(0, model.cfg.vocab_size, (2, 32), generator=g)
        loss = model(ids, labels=ids)
        opt.zero_grad()
        loss.backward()
        opt.step()
        ref.append(float(loss))
    for r in run_dist(_case_ring_llama, 2, mode):
        for a, b in zip(r["losses"], ref):
            assert abs(a - b) < 1e-4 * max(1.0, abs(b)), (r["losses"], ref)


@pytest.mark.gpu
def test_ring_pairs_on_hip_flash_kernels():
    """The per-pair HIP flash forward (with LSE) + LSE merge, and the per-pair HIP backward fed the
    merged output / LSE, reproduce full causal attention over the concatenated chunks (the ring
    simulated in one process: the kernels are the part a gloo run cannot exercise)."""
    from shuffle_exchange_amd.ops import native
    import importlib
    ra = importlib.import_module("shuffle_exchange_amd.sequence.ring_attention")
    native.require_hip()
    torch.manual_seed(0)
    p, Sl, B, H, Hk, D = 3, 128, 1, 4, 2, 128
    dev, bf = "cuda", torch.bfloat16
    q, k, v = (torch.randn(B, p * Sl, h, D, device=dev, dtype=bf) for h in (H, Hk, Hk))
    dy = torch.randn(B, p * Sl, H, D, device=dev, dtype=bf)
    qr, kr, vr = (t.float().requires_grad_() for t in (q, k, v))
    ref = _full(qr, kr, vr, True)
    ref.backward(dy.float())
    ch = lambda t, i: t[:, i * Sl:(i + 1) * Sl].contiguous()  # noqa: E731
    scale = D ** -0.5
    assert ra._hip_ok(ch(q, 0), ch(k, 0), ch(v, 0))
    outs, lses = [], []
    for i in range(p):
        o_acc = l_acc = None
        for j in range(i + 1):
            o, l = ra._pair_fwd(ch(q, i), ch(k, j), ch(v, j), j == i, scale)
            o_acc, l_acc = ra._merge(o_acc, l_acc, o, l)
        outs.append(o_acc.to(bf))
        lses.append(l_acc)
    out = torch.cat(outs, 1)
    assert ((out.float() - ref).norm() / ref.norm()).item() < 1e-2
    dq = torch.zeros_like(q, dtype=torch.float32)
    dk = torch.zeros_like(k, dtype=torch.float32)
    dv = torch.zeros_like(v, dtype=torch.float32)
    for i in range(p):
        for j in range(i + 1):
            a, b, c = ra._pair_bwd(ch(dy, i), ch(q, i), ch(k, j), ch(v, j), outs[i], lses[i], j == i, scale)
            dq[:, i * Sl:(i + 1) * Sl] += a
            dk[:, j * Sl:(j + 1) * Sl] += b
            dv[:, j * Sl:(j + 1) * Sl] += c
    for got, want in ((dq, qr.grad), (dk, kr.grad), (dv, vr.grad)):
        assert ((got - want).norm() / want.norm()).item() < 2e-2
