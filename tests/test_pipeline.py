"""Pipeline parallelism on gloo: 1F1B schedule shape, partitioning, and PipelineEngine training ==
the same layers trained sequentially in one process (pp=2 / pp=2 x dp=2 / pp=4, tied embeddings,
ZeRO-1 + fp32 / bf16-free CPU path)."""
import pytest
import torch

from .dist_utils import run_dist


def test_train_schedule_1f1b_counts():
    from shuffle_exchange_amd.runtime.pipe import schedule as S
    for stages in (1, 2, 4):
        for sid in range(stages):
            for M in (1, 3, 8):
                order = S.TrainSchedule(M, stages, sid).order()
                assert [m for k, m in order if k == "F"] == list(range(M))
                assert [m for k, m in order if k == "B"] == list(range(M))
                # a micro-batch's backward comes after its forward; in-flight never exceeds stages - sid
                live, peak = set(), 0
                for k, m in order:
                    (live.add if k == "F" else live.discard)(m)
                    peak = max(peak, len(live))
                assert peak <= max(1, min(stages - sid, M))


def test_partition_balanced():
    from shuffle_exchange_amd.runtime.pipe.module import partition_balanced, partition_uniform
    assert partition_uniform(10, 3) == [0, 4, 7, 10]
    parts = partition_balanced([1, 1, 10, 1, 1, 1], 3)
    assert parts[0] == 0 and parts[-1] == 6
    sizes = [sum([1, 1, 10, 1, 1, 1][parts[i]:parts[i + 1]]) for i in range(3)]
    assert max(sizes) == 10


def _layers(cfg):
    from shuffle_exchange_amd.models.llama_pipe import llama_pipeline_layers
    return llama_pipeline_layers(cfg)


def _case_pipe(rank, world, pp, steps, M, mbs, tie, zero_stage):
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.models import llama_config
    from shuffle_exchange_amd.models.llama_pipe import llama_pipe_loss
    from shuffle_exchange_amd.runtime.pipe.module import PipelineModule, TiedLayerSpec
    cfg = llama_config("llama-tiny", num_hidden_layers=4, tie_word_embeddings=tie)
    specs = _layers(cfg)
    pm = PipelineModule(specs, num_stages=pp, loss_fn=llama_pipe_loss, seed_layers=True, base_seed=77,
                        partition_method="uniform")
    ds = {"train_micro_batch_size_per_gpu": mbs, "gradient_accumulation_steps": M,
          "zero_optimization": {"stage": zero_stage}, "optimizer": {"type": "SGD", "params": {"lr": 0.1}}}
    eng, _, _, _ = sxe.initialize(model=pm, config=ds)
    dp, dpr = pm.mpu().get_data_parallel_world_size(), pm.mpu().get_data_parallel_rank()
    g = torch.Generator().manual_seed(5)
    batches = [torch.randint(0, cfg.vocab_size, (dp * M * mbs, 16), generator=g) for _ in range(steps)]
    losses = []
    for b in batches:
        mine = b.view(dp, M, mbs, 16)[dpr]
        it = iter([(mine[i], mine[i]) for i in range(M)])
        losses.append(float(eng.train_batch(it)))

    # sequential reference of the full layer stack, identical seeds, all 2*M micro-batches
    torch.manual_seed(0)
    ref_layers, tied = [], {}
    for i, s in enumerate(specs):
        torch.manual_seed(77 + i)
        if isinstance(s, TiedLayerSpec):
            if s.key not in tied:
                tied[s.key] = s.build()
            mod = tied[s.key]
            ref_layers.append((mod, s.forward_fn))
        else:
            ref_layers.append((s.build(), None))
    mods = torch.nn.ModuleList({id(m): m for m, _ in ref_layers}.values())
    opt = torch.optim.SGD(mods.parameters(), lr=0.1)
    ref_losses = []
    for b in batches:
        opt.zero_grad()
        tot = 0.0
        mbs_all = b.view(dp * M, mbs, 16)
        for x in mbs_all:
            h = x
            for m, fn in ref_layers:
                h = fn(m, h) if fn is not None else m(h)
            loss = llama_pipe_loss(h, x) / (dp * M)
            loss.backward()
            tot += float(loss)
        opt.step()
        ref_losses.append(tot)
    # compare this stage's layers with the reference layers of the same global index
    ok = True
    worst = 0.0
    for local_i, f in enumerate(pm.forward_funcs):
        gi = pm._local_start + local_i
        mod = f.args[0] if hasattr(f, "func") else f
        ref_mod = ref_layers[gi][0]
        for (n, p), (_, q) in zip(mod.named_parameters(), ref_mod.named_parameters()):
            d = (p.detach() - q.detach()).abs().max().item()
            worst = max(worst, d)
            ok = ok and d < 2e-5
    return {"losses": losses, "ref": ref_losses, "ok": ok, "worst": worst}


@pytest.mark.parametrize("world,pp,tie,zero", [(2, 2, False, 0), (4, 2, False, 1), (4, 4, True, 0), (2, 2, True, 1)])
def test_pipeline_matches_sequential(world, pp, tie, zero):
    res = run_dist(_case_pipe, world, pp, 2, 3, 2, tie, zero)
    for r in res:
        assert r["ok"], r["worst"]
        for a, b in zip(r["losses"], r["ref"]):
            assert a == pytest.approx(b, rel=1e-4)
