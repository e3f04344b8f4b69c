"""ZeRO user API pieces: OnDevice (meta / dtype construction), TiledLinear (== Linear, tiles are
separate ZeRO-3 fetch units), register_external_parameter, see_memory_usage, runtime utils."""
import torch

from .dist_utils import run_dist


def test_on_device_meta_and_dtype():
    import shuffle_exchange_amd as sxe
    with sxe.OnDevice(dtype=torch.bfloat16, device="meta"):
        m = torch.nn.Linear(8, 4)
    assert m.weight.is_meta and m.weight.dtype == torch.bfloat16
    with sxe.OnDevice(dtype=torch.float64, device="cpu"):
        m = torch.nn.Linear(8, 4)
    assert m.weight.device.type == "cpu" and m.weight.dtype == torch.float64
    assert torch.get_default_dtype() == torch.float32


def test_tiled_linear_matches_linear():
    from shuffle_exchange_amd.zero import TiledLinear, TiledLinearReturnBias
    torch.manual_seed(0)
    ref = torch.nn.Linear(13, 11)
    t = TiledLinear(13, 11, in_splits=3, out_splits=2, init_linear=ref)
    x = torch.randn(4, 13)
    assert torch.allclose(t(x), ref(x), atol=1e-6)
    tb = TiledLinearReturnBias(13, 11, in_splits=2, out_splits=3, init_linear=ref)
    y, b = tb(x)
    assert torch.allclose(y + b, ref(x), atol=1e-6)


def _case_tiled_zero3(rank, world):
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.zero import TiledLinear
    torch.manual_seed(0)
    model = torch.nn.Sequential(TiledLinear(16, 24, in_splits=2, out_splits=3), torch.nn.ReLU(), torch.nn.Linear(24, 4))
    ds = {"train_micro_batch_size_per_gpu": 2, "zero_optimization": {"stage": 3, "stage3_param_persistence_threshold": 0},
          "optimizer": {"type": "SGD", "params": {"lr": 0.1}}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(world * 2, 16, generator=g)
    y = torch.randn(world * 2, 4, generator=g)
    loss = ((eng(x[rank * 2:rank * 2 + 2]) - y[rank * 2:rank * 2 + 2]) ** 2).mean()
    eng.backward(loss)
    eng.step()
    from ._dist_cases import full_params
    return {"n_fg": len(eng.optimizer.fgroups), "params": full_params(eng)}


def test_tiled_linear_tiles_are_zero3_units():
    res = run_dist(_case_tiled_zero3, 2)
    from shuffle_exchange_amd.zero import TiledLinear
    torch.manual_seed(0)
    model = torch.nn.Sequential(TiledLinear(16, 24, in_splits=2, out_splits=3), torch.nn.ReLU(), torch.nn.Linear(24, 4))
    g = torch.Generator().manual_seed(5)
    x = torch.randn(4, 16, generator=g)
    y = torch.randn(4, 4, generator=g)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    ((model(x) - y) ** 2).mean().backward()
    opt.step()
    for r in res:
        assert r["n_fg"] >= 6 + 1  # six tiles + the plain Linear
        for n, p in model.named_parameters():
            assert torch.allclose(r["params"][n], p.detach(), atol=1e-6), n


def test_runtime_utils():
    from shuffle_exchange_amd.runtime.utils import partition_balanced, partition_uniform, see_memory_usage
    see_memory_usage("probe", force=True)
    assert partition_uniform(10, 3) == [0, 4, 7, 10]
    parts = partition_balanced([1, 1, 1, 10, 1, 1], 3)
    assert parts[0] == 0 and parts[-1] == 6 and len(parts) == 4
    loads = [sum([1, 1, 1, 10, 1, 1][parts[i]:parts[i + 1]]) for i in range(3)]
    assert max(loads) == 10


def _case_fp16_wrappers(rank, world):
    import shuffle_exchange_amd as sxe  # noqa: F401
    from shuffle_exchange_amd.runtime.fp16.fused_optimizer import BF16_Optimizer, FP16_Optimizer
    from shuffle_exchange_amd.parallel import groups
    groups.initialize()
    out = {}
    for name, make in (("fp16", lambda o: FP16_Optimizer(o, static_loss_scale=1.0)),
                       ("bf16", lambda o: BF16_Optimizer(o))):
        torch.manual_seed(0)
        m = torch.nn.Linear(8, 4)
        opt = make(torch.optim.SGD(m.parameters(), lr=0.1))
        x = torch.randn(4, 8, generator=torch.Generator().manual_seed(rank))
        opt.backward_prologue()
        m(x).pow(2).mean().backward()
        opt.reduce_gradients()
        opt.step()
        out[name] = m.weight.detach().clone()
    return out


def test_fp16_bf16_optimizer_wrappers():
    res = run_dist(_case_fp16_wrappers, 2)
    torch.manual_seed(0)
    m = torch.nn.Linear(8, 4)
    opt = torch.optim.SGD(m.parameters(), lr=0.1)
    xs = [torch.randn(4, 8, generator=torch.Generator().manual_seed(r)) for r in range(2)]
    (sum(m(x).pow(2).mean() for x in xs) / 2).backward()
    opt.step()
    for r in res:
        for k in ("fp16", "bf16"):
            assert torch.allclose(r[k], m.weight.detach(), atol=1e-6), k
