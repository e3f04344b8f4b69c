"""Ulysses sequence parallelism on gloo: the all-to-all layout transforms, DistributedAttention ==
full attention, and a Llama training step with SP=2 == the single-process step on full sequences."""
import pytest
import torch

from .dist_utils import run_dist


def _case_seq_head_roundtrip(rank, world):
    from shuffle_exchange_amd.parallel import groups
    from shuffle_exchange_amd.sequence.layer import head_to_seq, seq_to_head
    groups.initialize(sequence_parallel_size=world)
    g = groups.get_sequence_parallel_group()
    torch.manual_seed(0)
    full = torch.randn(2, 8 * world, 4 * world, 16)  # identical on all ranks
    local = full.chunk(world, dim=1)[rank]
    heads = seq_to_head(local, g)
    expect = full.chunk(world, dim=2)[rank]
    back = head_to_seq(heads, g)
    return {"ok_fwd": bool(torch.equal(heads, expect)), "ok_back": bool(torch.equal(back, local))}


def test_seq_head_all_to_all():
    for r in run_dist(_case_seq_head_roundtrip, 2):
        assert r["ok_fwd"] and r["ok_back"]


def _case_sp_train(rank, world, stage):
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    from shuffle_exchange_amd.parallel import groups
    from shuffle_exchange_amd.sequence.data import shard_batch_for_sp
    torch.manual_seed(0)
    cfg = llama_config("llama-tiny", sequence_parallel=True)
    model = LlamaForCausalLM(cfg)
    ds = {"train_micro_batch_size_per_gpu": 2, "sequence_parallel_size": world,
          "zero_optimization": {"stage": stage}, "optimizer": {"type": "SGD", "params": {"lr": 0.1}}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    g = torch.Generator().manual_seed(11)
    losses = []
    for _ in range(2):
        ids = torch.randint(0, cfg.vocab_size, (2, 32), generator=g)
        b = shard_batch_for_sp(ids, groups.get_sequence_parallel_rank(), world)
        loss = eng(b["input_ids"], labels=b["labels"], position_ids=b["position_ids"], shift_labels=False)
        from shuffle_exchange_amd import comm
        tot = loss.detach().clone()
        comm.all_reduce(tot, group=groups.get_sequence_parallel_group())
        eng.backward(loss)
        eng.step()
        losses.append(float(tot))
    from ._dist_cases import full_params
    return {"losses": losses, "params": full_params(eng)}


def _reference_full_seq():
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    torch.manual_seed(0)
    model = LlamaForCausalLM(llama_config("llama-tiny"))
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    g = torch.Generator().manual_seed(11)
    losses = []
    for _ in range(2):
        ids = torch.randint(0, 512, (2, 32), generator=g)
        loss = model(ids, labels=ids)
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(float(loss))
    return {"losses": losses, "params": {n: p.detach().clone() for n, p in model.named_parameters()}}


@pytest.mark.parametrize("stage", [1, 3])
def test_ulysses_sp_matches_full_sequence(stage):
    res = run_dist(_case_sp_train, 2, stage)
    ref = _reference_full_seq()
    for r in res:
        for a, b in zip(r["losses"], ref["losses"]):
            assert a == pytest.approx(b, rel=1e-5)
        for k, v in ref["params"].items():
            assert torch.allclose(r["params"][k], v, atol=2e-5), k
