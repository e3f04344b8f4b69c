"""ZeRO-0/1/2/3 and Shuffle-exchange on CPU with gloo (multi-process), against single-process
PyTorch references. Oracles: ZeRO == single-process AdamW on the global batch;
RR(SGD) == DP-SGD; H-RR == RR; shuffle groups rank-consistent; Gossip mass conserved;
checkpoint round trip; collective fingerprints."""
import pytest
import torch

from . import _dist_cases as C
from .dist_utils import run_dist


def _close(a, b, tol=2e-5):
    for k in b:
        d = (a[k] - b[k]).abs().max().item()
        scale = b[k].abs().max().item() + 1e-6
        assert d <= tol * max(1.0, scale), f"{k}: max diff {d}"


ADAMW = {"type": "AdamW", "params": {"lr": 1e-2, "weight_decay": 0.01}}


@pytest.mark.parametrize("stage", [0, 1, 2, 3])
def test_zero_matches_single_process_adamw(stage):
    world, mbs, seq, steps = 2, 2, 16, 3
    ds = {"train_micro_batch_size_per_gpu": mbs, "zero_optimization": {"stage": stage,
                                                                       "stage3_param_persistence_threshold": 0},
          "optimizer": ADAMW}
    res = run_dist(C.case_train, world, ds, steps, mbs, seq)
    ref = C.reference_train(ADAMW, steps, world, mbs, seq)
    for r in res:
        # Adam normalises each element by its own gradient scale: a near-zero gradient summed in a
        # different order (2-rank reduce vs one process) moves its update by up to a fraction of lr
        _close(r["params"], ref, tol=1e-4)


def test_zero2_grad_accumulation_and_clipping():
    world, mbs, seq, steps = 2, 1, 16, 2
    ds = {"train_micro_batch_size_per_gpu": mbs, "gradient_accumulation_steps": 1, "gradient_clipping": 0.05,
          "zero_optimization": {"stage": 2}, "optimizer": ADAMW}
    res = run_dist(C.case_train, world, ds, steps, mbs, seq)
    ref = C.reference_train(ADAMW, steps, world, mbs, seq, clip=0.05)
    for r in res:
        _close(r["params"], ref, tol=1e-4)


SGD = {"type": "SGD", "params": {"lr": 0.05}}


@pytest.mark.parametrize("method,stage", [("RR", 2), ("RR", 1), ("H-RR", 2), ("RR", 3)])
def test_shuffle_exchange_rr_equals_dp_sgd(method, stage):
    """Averaging the bit16 iterate across slices after each SGD step equals DP-SGD over all ranks."""
    world, mbs, seq, steps = 4, 1, 16, 3
    ds = {"train_micro_batch_size_per_gpu": mbs,
          "zero_optimization": {"stage": stage, "stage3_param_persistence_threshold": 0}, "optimizer": SGD}
    res = run_dist(C.case_train, world, ds, steps, mbs, seq, {"method": method, "slice_count": 2})
    ref = C.reference_train(SGD, steps, world, mbs, seq)
    for r in res:
        _close(r["params"], ref, tol=1e-5)


@pytest.mark.parametrize("method", ["RR", "H-RR"])
def test_shuffle_exchange_with_offload_param_equals_dp_sgd(method):
    """ZeRO-3 offload_param keeps the bit16 shards in (pinned) host memory: the inter-slice average
    runs on them through the pack buffer and still equals DP-SGD over all ranks."""
    world, mbs, seq, steps = 4, 1, 16, 3
    ds = {"train_micro_batch_size_per_gpu": mbs, "optimizer": SGD,
          "zero_optimization": {"stage": 3, "stage3_param_persistence_threshold": 0,
                                "offload_param": {"device": "cpu"}}}
    res = run_dist(C.case_train, world, ds, steps, mbs, seq, {"method": method, "slice_count": 2})
    ref = C.reference_train(SGD, steps, world, mbs, seq)
    for r in res:
        _close(r["params"], ref, tol=1e-5)


def test_shuffle_groups_consistent_and_reshuffle():
    world = 4
    res = run_dist(C.case_shuffle_groups, world, 1, 2, 2, 6)
    n_calls = len(res[0])
    changed = False
    for t in range(n_calls):
        groups_at_t = [frozenset(r[t]) for r in res]
        for rank, g in enumerate(groups_at_t):
            assert rank in g and len(g) == 2
            for other in g:
                assert groups_at_t[other] == g  # membership agreed by every member
        if t > 0 and groups_at_t != [frozenset(r[t - 1]) for r in res]:
            changed = True
        if t % 2 == 1:  # shuffle_step = 2 -> groups only change on even call counts
            assert groups_at_t == [frozenset(r[t - 1]) for r in res]
    assert changed or n_calls < 3


def test_gossip_mass_and_synchronization():
    world = 4
    res = run_dist(C.case_gossip, world, 3)
    for r in res:
        assert abs(r["mass"] - 1.0) < 1e-5
    for r in res[1:]:
        _close(r["params"], res[0]["params"], tol=1e-6)


@pytest.mark.parametrize("stage", [2, 3])
def test_checkpoint_roundtrip(stage, tmp_path):
    res = run_dist(C.case_ckpt, 2, stage, str(tmp_path), 2, 2)
    for r in res:
        assert r["client"] == 7
        assert r["lr"] == pytest.approx(r["lr_ref"])
        for a, b in zip(r["cont"], r["resumed"]):
            assert a == pytest.approx(b, rel=1e-5, abs=1e-6)
    files = res[0]["files"]
    assert any(f.startswith("zero_pp_rank_0_mp_rank_00") and f.endswith("optim_states.pt") for f in files)
    assert any(f.startswith("zero_pp_rank_1_mp_rank_00") and f.endswith("optim_states.pt") for f in files)
    if stage == 3:
        assert "zero_pp_rank_0_mp_rank_00_model_states.pt" in files
    else:
        assert "mp_rank_00_model_states.pt" in files


def test_collectives_and_fingerprint():
    world = 2
    res = run_dist(C.case_collectives, world)
    for r, out in enumerate(res):
        assert out["ar"] == [3.0] * 8
        assert out["ag"] == [0.0] * 4 + [1.0] * 4
        assert out["rs"] == [2 * (2 * r), 2 * (2 * r + 1)]
        assert out["a2a"] == [0.0, 1.0]
        assert out["fp_ok"]
    res = run_dist(C.case_fingerprint_mismatch, world)
    assert res == ["mismatch-detected"] * world


@pytest.mark.parametrize("knobs,tol", [({"zero_quantized_weights": True}, 5e-2),
                                       ({"zero_quantized_gradients": True}, 5e-2),
                                       ({"zero_quantized_gradients": True,
                                         "zeropp_loco_param": {"err_beta": 0.8, "reset_T": 2}}, 5e-2),
                                       ({"zero_hpz_partition_size": 2}, 1e-5)])
def test_zeropp_matches_zero3(knobs, tol):
    """ZeRO++ qwZ / qgZ (int8, with and without LoCo error feedback) track plain ZeRO-3 closely; hpZ
    (secondary intra-group shards) is exact."""
    world, mbs, seq, steps = 4, 1, 16, 3
    base = {"stage": 3, "stage3_param_persistence_threshold": 0}
    SGD = {"type": "SGD", "params": {"lr": 0.05}}
    ds = {"train_micro_batch_size_per_gpu": mbs, "zero_optimization": dict(base, **knobs), "optimizer": SGD}
    ref_ds = {"train_micro_batch_size_per_gpu": mbs, "zero_optimization": base, "optimizer": SGD}
    res = run_dist(C.case_train, world, ds, steps, mbs, seq)
    ref = run_dist(C.case_train, world, ref_ds, steps, mbs, seq)
    for a, b in zip(res[0]["losses"], ref[0]["losses"]):
        assert abs(a - b) <= tol * abs(b)
    for k, v in ref[0]["params"].items():
        d = (res[0]["params"][k] - v).norm() / (v.norm() + 1e-12)
        assert d < tol, (k, float(d))


def _case_offload_states(rank, world, stage):
    import shuffle_exchange_amd as sxe
    model, cfg = C.tiny_llama(0)
    ds = {"train_micro_batch_size_per_gpu": 1, "zero_optimization": {"stage": stage,
                                                                     "stage3_param_persistence_threshold": 0},
          "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    batches = C.global_batches(cfg, world, 1, 16, 4)

    def run(bs):
        for b in bs:
            local = b[rank:rank + 1]
            loss = eng(local, labels=local)
            eng.backward(loss)
            eng.step()
    run(batches[:2])
    eng.offload_states()
    eng.reload_states()
    run(batches[2:])
    return C.full_params(eng)


@pytest.mark.parametrize("stage", [1, 3])
def test_offload_reload_states_roundtrip(stage):
    a = run_dist(_case_offload_states, 2, stage)
    b = run_dist(C.case_train, 2, {"train_micro_batch_size_per_gpu": 1,
                                   "zero_optimization": {"stage": stage, "stage3_param_persistence_threshold": 0},
                                   "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}}}, 4, 1, 16)
    _close(a[0], b[0]["params"], tol=1e-6)


def test_zero3_reuse_distance_skips_backward_gathers():
    """stage3_max_reuse_distance (reference partitioned_param_coordinator.py:529-559): units whose
    forward->backward reuse distance fits the budget stay gathered, so the backward all-gathers
    disappear; the numerics are unchanged (== single-process AdamW)."""
    world, mbs, seq, steps = 2, 2, 16, 3
    keep = run_dist(C.case_zero3_reuse, world, 10**12, steps, mbs, seq)
    drop = run_dist(C.case_zero3_reuse, world, 0, steps, mbs, seq)
    ref = C.reference_train(ADAMW, steps, world, mbs, seq)
    for r in keep + drop:
        _close(r["params"], ref, tol=1e-4)
    assert keep[0]["gathers"] < drop[0]["gathers"], (keep[0]["gathers"], drop[0]["gathers"])


def test_zero3_tied_embeddings_external_parameter():
    res = run_dist(C.case_tied_zero3, 2, 2)
    model, cfg = C.tiny_llama(0, tie_word_embeddings=True)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    for b in C.global_batches(cfg, 2, 1, 16, 2):
        loss = model(b, labels=b)
        opt.zero_grad()
        loss.backward()
        opt.step()
    ref = {n: p.detach().clone() for n, p in model.named_parameters()}
    for r in res:
        assert "lm_head#external" in r["fgs"]
        _close(r["params"], ref)


def test_zero3_deferred_reduce_scatter_matches_per_microstep():
    """stage3_defer_reduce: one reduce-scatter per unit per optimizer step (not per micro-step),
    same parameters as reducing every micro-step."""
    world, steps, mbs, gas, seq = 2, 2, 2, 3, 16
    d = run_dist(C.case_zero3_defer, world, True, steps, mbs, gas, seq)
    n = run_dist(C.case_zero3_defer, world, False, steps, mbs, gas, seq)
    assert d[0]["defer"] and not n[0]["defer"]
    assert n[0]["rs"] == gas * d[0]["rs"], (n[0]["rs"], d[0]["rs"])
    for k, v in n[0]["params"].items():
        torch.testing.assert_close(d[0]["params"][k], v, atol=1e-4, rtol=1e-3)  # Adam amplifies sum order


def test_zero3_retain_params_in_step_gathers_once_per_step():
    """stage3_retain_params_in_step: gathered units stay resident across the micro-steps of one
    optimizer step -> one all-gather per unit per step; same parameters."""
    world, steps, mbs, gas, seq = 2, 2, 2, 3, 16
    r = run_dist(C.case_zero3_defer, world, True, steps, mbs, gas, seq, True)
    n = run_dist(C.case_zero3_defer, world, True, steps, mbs, gas, seq, False)
    assert r[0]["ag"] <= steps * (r[0]["n_units"] + 1), (r[0]["ag"], r[0]["n_units"])
    assert n[0]["ag"] >= 2 * r[0]["ag"], (n[0]["ag"], r[0]["ag"])  # 16 vs 6 per step at gas 3
    for k, v in n[0]["params"].items():
        torch.testing.assert_close(r[0]["params"][k], v, atol=1e-6, rtol=1e-5)


@pytest.mark.parametrize("world", [2, 4])
def test_zero_init_partitions_at_construction(world):
    """zero.Init: per-rank construction memory is ~full/W + one module, ranks agree on the weights
    even with different seeds, GatheredParameters(modifier_rank=0) edits propagate, and ZeRO-3
    trains from the partitioned model (reference partition_parameters.py:1141, :1109-1116)."""
    layers = 4
    res = run_dist(C.case_zero_init, world, layers, 2)
    r0 = res[0]
    st = r0["stats"]
    full = r0["full_numel"]
    assert r0["empty"] and r0["left"] == 0
    # one module's own parameters whole at a time: the largest is a decoder layer or the embedding
    assert st["peak_full_numel"] <= max(r0["layer_numel"], r0["emb_numel"])
    assert st["peak_full_numel"] < full / 2
    for r in res:
        assert abs(r["stats"]["partition_numel"] - full / world) <= 64 * st["params"]
    for r in res[1:]:
        for k in r0["before"]:
            assert torch.equal(r["before"][k], r0["before"][k]), k
            assert torch.allclose(r["after"][k], r0["after"][k], atol=1e-6), k
    assert torch.all(r0["before"]["norm.weight"] == 1.5)
    assert all(l == l for l in r0["losses"])
    # world-size invariant: every weight was initialised whole (by its constructor) on rank 0 and
    # broadcast, so the partitioned model equals the unpartitioned one built from rank 0's seed
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    torch.manual_seed(100)
    ref = LlamaForCausalLM(llama_config("llama-tiny", num_hidden_layers=layers))
    for n, p in ref.named_parameters():
        if n != "norm.weight":
            assert torch.equal(r0["before"][n], p.detach().float()), n


def test_broadcast_coalesced_in_place_and_bucketed():
    res = run_dist(C.case_broadcast_coalesced, 2)
    for r in res:
        assert r["ok"]
    # 5000 doubles (40 KB) and the non-contiguous one go alone; the 1000+10+7 floats share a bucket
    assert res[0]["n"] == 3


@pytest.mark.parametrize("stage,se", [(0, None), (2, None), (3, None), (2, {"method": "RR", "slice_count": 2}),
                                      (1, {"method": "H-RR", "slice_count": 1})])
def test_one_step_metadata_collective_per_step(stage, se):
    """Gradient norm and the world-wide overflow flag travel in ONE all-reduce per optimizer step
    (the reference issues a norm all-reduce per group plus a separate overflow all-reduce)."""
    steps = 3
    res = run_dist(C.case_step_meta, 4, stage, se, steps)
    for counts in res:
        assert counts.get("step_meta", 0) == steps, counts
        if se is None:
            assert counts.get("all_reduce", 0) == (0 if stage else counts.get("all_reduce", 0)), counts


def test_moe_zero0_clipping_keeps_dense_weights_in_sync():
    a, b = run_dist(C.case_mixtral_dense_sync, 2)
    for k in a:
        assert torch.allclose(a[k], b[k], atol=1e-6), k


class _EmbNet(torch.nn.Module):
    def __init__(self, sparse):
        super().__init__()
        torch.manual_seed(0)
        self.emb = torch.nn.Embedding(1000, 16, sparse=sparse)
        self.out = torch.nn.Linear(16, 4)

    def forward(self, ids):
        return self.out(self.emb(ids)).pow(2).mean()


def _case_sparse(rank, world, sparse):
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd import comm as dist
    model = _EmbNet(sparse)
    ds = {"train_micro_batch_size_per_gpu": 4, "gradient_accumulation_steps": 2, "sparse_gradients": sparse,
          "zero_optimization": {"stage": 0}, "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    calls = {"ag": 0}
    orig = dist.all_gather_into_tensor

    def ag(*a, **k):
        calls["ag"] += 1
        return orig(*a, **k)
    dist.all_gather_into_tensor = ag
    g = torch.Generator().manual_seed(5)
    for _ in range(6):
        ids = torch.randint(0, 50, (world * 4, 7), generator=g)[rank * 4:(rank + 1) * 4]  # few rows touched
        loss = eng(ids)
        eng.backward(loss)
        eng.step()
    dist.all_gather_into_tensor = orig
    return {"params": [p.detach().clone() for p in eng.module.parameters()], "ag": calls["ag"]}


def test_sparse_embedding_gradients_stage0():
    """sparse_gradients with nn.Embedding(sparse=True): the touched rows are all-gathered (reference
    engine.py sparse_allreduce) and training equals the dense-gradient run."""
    sp = run_dist(_case_sparse, 2, True)
    dn = run_dist(_case_sparse, 2, False)
    assert sp[0]["ag"] > 0 and dn[0]["ag"] == 0
    for a, b in zip(sp[0]["params"], dn[0]["params"]):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    for a, b in zip(sp[0]["params"], sp[1]["params"]):
        assert torch.equal(a, b)


class _TiedEmbNet(torch.nn.Module):
    """Sparse embedding tied to the output projection: its gradient is sparse + dense = dense."""

    def __init__(self, sparse):
        super().__init__()
        torch.manual_seed(0)
        self.emb = torch.nn.Embedding(64, 16, sparse=sparse)

    def forward(self, ids):
        h = self.emb(ids)
        return (h @ self.emb.weight.t()).pow(2).mean()


def _case_tied_sparse(rank, world, sparse):
    import shuffle_exchange_amd as sxe
    model = _TiedEmbNet(sparse)
    ds = {"train_micro_batch_size_per_gpu": 4, "gradient_accumulation_steps": 2, "sparse_gradients": sparse,
          "zero_optimization": {"stage": 0}, "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    g = torch.Generator().manual_seed(5)
    for _ in range(4):
        ids = torch.randint(0, 64, (world * 4, 7), generator=g)[rank * 4:(rank + 1) * 4]
        loss = eng(ids)
        eng.backward(loss)
        eng.step()
    return [p.detach().clone() for p in eng.module.parameters()]


def test_sparse_marked_weight_with_dense_gradient_stays_in_sync():
    """A sparse-marked weight that receives a dense gradient is reduced densely: replicas stay
    identical and equal the dense run (the dense part was never reduced before)."""
    sp = run_dist(_case_tied_sparse, 2, True)
    dn = run_dist(_case_tied_sparse, 2, False)
    for a, b in zip(sp[0], sp[1]):
        assert torch.equal(a, b)
    for a, b in zip(sp[0], dn[0]):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def test_zero3_reduce_scatter_has_its_own_communicator_and_one_refresh_gather():
    """ZeRO-3's gradient reduce-scatter runs on a second communicator over the slice ranks (RCCL
    serialises every collective of one communicator, so the backward prefetch all-gathers would
    queue it), and the post-step rebuild of the persistent units is ONE packed all-gather; the
    trained parameters still match the reference."""
    world, steps = 2, 2
    for r in run_dist(C.case_zero3_comm_design, world, steps):
        assert not r["same_group"]
        assert r["rs_ranks"] == r["ag_ranks"] == [0, 1]
        assert r["n_persist"] > 1
        assert r["refresh"] == [1] * steps, r["refresh"]
    ref = C.reference_train({"type": "SGD", "params": {"lr": 0.1}}, steps, world, 1, 16)
    _close(r["params"], ref)


class _Branchy(torch.nn.Module):
    """Parameter `b` only gets a gradient on odd steps (a MoE expert that received no tokens)."""

    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(8, 8)
        self.b = torch.nn.Linear(8, 8)
        self.use_b = False

    def forward(self, x):
        y = self.a(x)
        return self.b(y) if self.use_b else y


def _case_stale(rank, world, stage, gas):
    import shuffle_exchange_amd as sxe
    torch.manual_seed(0)
    m = _Branchy()
    ref = _Branchy()
    ref.load_state_dict(m.state_dict())
    ds = {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": gas, "gradient_clipping": 1.0,
          "zero_optimization": {"stage": stage}, "optimizer": ADAMW}
    eng, _, _, _ = sxe.initialize(model=m, config=ds)
    opt = torch.optim.AdamW(ref.parameters(), lr=1e-2, weight_decay=0.01)
    for p in ref.parameters():  # a missing gradient is a zero gradient (flat ZeRO semantics)
        p.grad = torch.zeros_like(p)
    g = torch.Generator().manual_seed(5)
    for step in range(4):
        m.use_b = ref.use_b = step % 2 == 1
        opt.zero_grad(set_to_none=False)
        for _ in range(gas):
            x = torch.randn(2, 8, generator=g)
            loss = eng(x).pow(2).mean()
            eng.backward(loss)
            eng.step()
            (ref(x).pow(2).mean() / gas).backward()
        torch.nn.utils.clip_grad_norm_(ref.parameters(), 1.0)
        opt.step()
    return {k: v.detach().clone() for k, v in m.state_dict().items()}, {k: v.detach().clone() for k, v in ref.state_dict().items()}


@pytest.mark.parametrize("stage,gas", [(1, 1), (1, 2), (2, 1), (2, 2)])
def test_single_rank_stale_accumulators(stage, gas):
    """ZeRO-1/2 on one rank mark the fp32 gradient accumulators stale after a step instead of
    zeroing them: the first write of the next step overwrites, and a parameter without a gradient
    in a step (here `b` on even steps) is zeroed before the update -- the trajectory equals torch
    AdamW fed zero gradients for the unused parameter."""
    got, ref = run_dist(_case_stale, 1, stage, gas)[0]
    _close(got, ref, tol=1e-4)
