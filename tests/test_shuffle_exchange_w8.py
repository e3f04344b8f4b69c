"""Shuffle-exchange at the target topology: 8 gloo ranks (one MI355X node's worth), slice_count 2
and 4, rings 2 and 4, ZeRO stages 1/2/3 -- checked against the exact averaging semantics of the
reference (runtime/zero/stage_1_and_2.py:205-250 groups, :692-734 shuffle/synchronization,
:2092-2250 the per-step exchange).

Every inter-slice exchange call is intercepted on every rank: a rank-specific offset is added to
the chunk first (so a wrong grouping cannot hide inside a small mean), the chunk is captured before
and after the real exchange, and the parent process checks, call by call:
  RR / H-RR    after == mean of `before` over all slices holding the same chunk offset;
  shuffle      after == mean over the CURRENT ring (the group the rank reported at that call), and
               the rings are redrawn exactly every `shuffle_step` shuffle_exchange() calls;
  Gossip       the push-sum merge of the next step == the hand-computed weighted average of the
               receiver's chunk and the sender's pushed chunk, with alphas replayed from the seeded
               generator (senders/destinations) -- over several steps;
  synchronization()  after == world mean over all slices.
fp32 models make the expected means exact; a separate bf16 case pins RR's rounding against the
fp32 mean (at most a few bf16 ulps: the slice count is a power of two, so the pre-division is
exact and only the summation rounds)."""
import pytest
import torch

from ._dist_cases import global_batches, tiny_llama
from .dist_utils import run_dist

W = 8


def _capture(se, log, slice_id):
    real_sync, real_pre = se.sync, se.pre_step

    def sync(shards, masters=None):
        for t in shards:
            t.add_(float(slice_id + 1))  # slice-specific: a wrong group gives a visibly wrong mean
        before = [t.detach().float().clone() for t in shards]
        groups = list(se.group_ranks) if se.group_ranks is not None else None
        real_sync(shards, masters)
        log.append({"kind": "sync", "before": before, "after": [t.detach().float().clone() for t in shards],
                    "group": groups})

    def pre_step(shards):
        before = [t.detach().float().clone() for t in shards]
        real_pre(shards)
        log.append({"kind": "pre", "before": before, "after": [t.detach().float().clone() for t in shards]})

    se.sync, se.pre_step = sync, pre_step


def _case(rank, world, runs):
    import shuffle_exchange_amd as sxe
    out = []
    for method, S, rings, stage, steps, bf16 in runs:
        model, cfg = tiny_llama(0)
        ds = {"train_micro_batch_size_per_gpu": 1, "zero_optimization": {"stage": stage,
                                                                          "stage3_param_persistence_threshold": 0},
              "optimizer": {"type": "SGD", "params": {"lr": 0.05}}}
        if bf16:
            ds["bf16"] = {"enabled": True}
        eng, _, _, _ = sxe.initialize(model=model, config=ds, method=method, slice_count=S, rings=rings,
                                      shuffle_step=2)
        se = eng.optimizer.se
        log, shuffles = [], []
        _capture(se, log, se.topo.slice_id)
        for b in global_batches(cfg, world, 1, 16, steps):
            local = b[rank:rank + 1]
            loss = eng(local, labels=local)
            eng.backward(loss)
            eng.step()
            eng.shuffle_exchange()
            shuffles.append(list(se.group_ranks) if se.group_ranks is not None else None)
        if method in ("shuffle", "Gossip"):
            real, cap = se.synchronization, {}

            def synchronization(sh):
                cap["before"] = [t.detach().float().clone() for t in sh]
                r = real(sh)
                cap["after"] = [t.detach().float().clone() for t in sh]
                return r
            se.synchronization = synchronization
            eng.synchronization()
            log.append({"kind": "world", "before": cap["before"], "after": cap["after"], "group": None})
        out.append({"log": log, "slice": se.topo.slice_id, "offset": se.topo.offset, "shuffles": shuffles,
                    "seed": se.seed, "n": se.topo.num_slices})
    return out


def _same_offset(res, k, r):
    return [q for q in range(W) if res[q][k]["offset"] == res[r][k]["offset"]]


def _mean(tensors):
    return torch.stack([t.double() for t in tensors]).mean(0).float()


def _check_means(res, k, group_of, tol):
    log0 = res[0][k]["log"]
    for c, entry in enumerate(log0):
        if entry["kind"] not in ("sync", "world"):
            continue
        for r in range(W):
            e = res[r][k]["log"][c]
            members = group_of(r, e)
            for i, after in enumerate(e["after"]):
                exp = _mean([res[q][k]["log"][c]["before"][i] for q in members])
                torch.testing.assert_close(after, exp, rtol=0, atol=tol, msg=lambda m: f"call {c} rank {r}: {m}")


RUNS = [("RR", 2, 8, 1, 2, False), ("RR", 4, 8, 2, 2, False), ("RR", 2, 8, 3, 2, False),
        ("H-RR", 2, 2, 2, 2, False), ("H-RR", 4, 2, 1, 2, False),
        ("shuffle", 2, 2, 2, 5, False), ("shuffle", 2, 4, 1, 3, False), ("shuffle", 2, 2, 3, 3, False),
        ("Gossip", 2, 8, 1, 3, False), ("Gossip", 4, 8, 2, 3, False),
        ("RR", 2, 8, 2, 1, True)]


@pytest.fixture(scope="module")
def w8():
    return run_dist(_case, W, RUNS)


@pytest.mark.parametrize("k", [i for i, r in enumerate(RUNS) if r[0] in ("RR", "H-RR") and not r[5]])
def test_rr_and_hrr_global_mean(w8, k):
    _check_means(w8, k, lambda r, e: _same_offset(w8, k, r), 1e-6)


@pytest.mark.parametrize("k", [i for i, r in enumerate(RUNS) if r[0] == "shuffle"])
def test_shuffle_ring_mean_and_reshuffle(w8, k):
    method, S, rings, stage, steps, _ = RUNS[k]
    n = W // S
    _check_means(w8, k, lambda r, e: e["group"] if e["group"] is not None else _same_offset(w8, k, r), 1e-6)
    for r in range(W):
        for e in w8[r][k]["log"]:
            if e["kind"] == "sync":
                assert r in e["group"] and len(e["group"]) == n // rings
    # the rings change only on every shuffle_step-th (=2nd) shuffle_exchange() call
    hist = [tuple(w8[0][k]["shuffles"][t]) for t in range(steps)]
    for t in range(1, steps):
        if (t + 1) % 2 == 1:
            assert hist[t] == hist[t - 1], (t, hist)
    # membership is agreed: every member of my ring reports the same ring
    for t in range(steps):
        for r in range(W):
            g = w8[r][k]["shuffles"][t]
            for q in g:
                assert sorted(w8[q][k]["shuffles"][t]) == sorted(g)


@pytest.mark.parametrize("k", [i for i, r in enumerate(RUNS) if r[0] in ("shuffle", "Gossip")])
def test_synchronization_is_world_mean(w8, k):
    log = w8[0][k]["log"]
    c = len(log) - 1
    assert log[c]["kind"] == "world"
    for r in range(W):
        e = w8[r][k]["log"][c]
        for i, after in enumerate(e["after"]):
            exp = _mean([w8[q][k]["log"][c]["before"][i] for q in _same_offset(w8, k, r)])
            torch.testing.assert_close(after, exp, rtol=0, atol=1e-6)


def _replay_gossip(seed, n, p, steps):
    """Senders / destinations per step from the seeded generator (ShuffleExchange._gossip)."""
    g = torch.Generator()
    g.manual_seed(seed)
    plan = []
    for _ in range(steps):
        senders = torch.bernoulli(torch.full((n,), p), generator=g).tolist()
        dests = torch.randint(0, n, (n,), generator=g).tolist()
        msgs = [(sid, int(dests[sid])) for sid in range(n) if senders[sid] == 1 and dests[sid] != sid]
        plan.append(msgs)
    return plan


@pytest.mark.parametrize("k", [i for i, r in enumerate(RUNS) if r[0] == "Gossip"])
def test_gossip_push_sum_merge(w8, k):
    method, S, rings, stage, steps, _ = RUNS[k]
    n = W // S
    plan = _replay_gossip(w8[0][k]["seed"], n, 1.0, steps)
    # push-sum mass of every slice through the steps: (alpha at merge start, [(alpha_msg, sender)])
    alpha = [1.0 / n] * n
    merges = []
    for t in range(steps - 1):
        inbox = {d: [] for d in range(n)}
        for sid, dest in plan[t]:  # sync of step t: the sender halves and pushes
            alpha[sid] /= 2
            inbox[dest].append((alpha[sid], sid))
        step_m = {}
        for d in range(n):  # merge at the start of step t+1 (reference stage_1_and_2.py:2092-2108)
            step_m[d] = (alpha[d], inbox[d])
            alpha[d] += sum(a for a, _ in inbox[d])
        merges.append(step_m)
    assert abs(sum(alpha) - 1.0) < 1e-12  # mass conserved
    for r in range(W):
        res_r = w8[r][k]
        me = res_r["slice"]
        syncs = [e for e in res_r["log"] if e["kind"] == "sync"]
        pres = [e for e in res_r["log"] if e["kind"] == "pre"]
        assert len(syncs) == steps and len(pres) == steps  # pres[0]: nothing queued yet
        for t in range(steps - 1):
            a, inbox = merges[t][me]
            pre = pres[t + 1]
            exp = [x.double() for x in pre["before"]]
            for am, sid in inbox:
                peer = next(q for q in range(W) if w8[q][k]["slice"] == sid and w8[q][k]["offset"] == res_r["offset"])
                sent = [e for e in w8[peer][k]["log"] if e["kind"] == "sync"][t]["before"]
                exp = [x * (a / (a + am)) + c.double() * (am / (a + am)) for x, c in zip(exp, sent)]
                a += am
            for got, e in zip(pre["after"], exp):
                torch.testing.assert_close(got, e.float(), rtol=0, atol=1e-5)
            if not inbox:  # no queued message -> the chunk is untouched
                for got, b in zip(pre["after"], pre["before"]):
                    assert torch.equal(got, b)


def test_rr_bf16_rounding_vs_fp32_mean(w8):
    """bf16 RR over 4 slices: within 4 bf16 ulps of the exact fp32 mean of the bf16 chunks."""
    k = next(i for i, r in enumerate(RUNS) if r[5])
    log = w8[0][k]["log"]
    for c, entry in enumerate(log):
        if entry["kind"] != "sync":
            continue
        for r in range(W):
            e = w8[r][k]["log"][c]
            for i, after in enumerate(e["after"]):
                exp = _mean([w8[q][k]["log"][c]["before"][i] for q in _same_offset(w8, k, r)])
                ulp = torch.ldexp(torch.ones_like(exp), torch.frexp(exp.abs().clamp_min(1e-30))[1] - 8)
                assert ((after - exp).abs() <= 4 * ulp).all(), (c, r, ((after - exp).abs() / ulp).max())


def _case_op_counts(rank, world, method, stage):
    """Collectives issued by one post-step inter-slice exchange with many flat units."""
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd import comm
    model, cfg = tiny_llama(0)
    ds = {"train_micro_batch_size_per_gpu": 1, "optimizer": {"type": "SGD", "params": {"lr": 0.05}},
          "zero_optimization": {"stage": stage, "reduce_bucket_size": 20000, "stage3_param_persistence_threshold": 0}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds, method=method, slice_count=2, rings=2, shuffle_step=2)
    b = global_batches(cfg, world, 1, 16, 1)[0][rank:rank + 1]
    eng.backward(eng(b, labels=b))
    se = eng.optimizer.se
    real = se.sync
    counts = {}

    def counted(shards, masters=None):
        comm.reset_comms_stats()
        real(shards, masters)
        counts.update(comm.get_op_counts())
        counts["chunks"] = len(shards)
    se.sync = counted
    eng.step()
    return counts


@pytest.mark.parametrize("method,stage", [("RR", 2), ("RR", 1), ("shuffle", 2), ("H-RR", 2)])
def test_inter_slice_exchange_is_one_collective_per_step(method, stage):
    """RR / shuffle: ONE all-reduce per step over all chunks packed together (not one per chunk);
    H-RR: one reduce + one broadcast (+ one all-reduce on the top ranks)."""
    res = run_dist(_case_op_counts, W, method, stage)
    for r, c in enumerate(res):
        assert c["chunks"] > 1, c  # several flat units: the packing is what keeps it at one call
        if method in ("RR", "shuffle"):
            assert c.get("all_reduce", 0) == 1, (r, c)
        else:
            assert c.get("reduce", 0) == 1 and c.get("broadcast", 0) == 1 and c.get("all_reduce", 0) <= 1, (r, c)
