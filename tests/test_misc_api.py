"""Smaller API pieces: muP optimizers, contiguous allocator, trace-range decorator, ZeRO-3 linear."""
import torch

from shuffle_exchange_amd.ops import optim
from shuffle_exchange_amd.runtime.lr_schedules import WarmupCosineLR, WarmupLR
from shuffle_exchange_amd.runtime.zero.contiguous_memory_allocator import ContiguousMemoryAllocator


def _mup_params():
    w = torch.nn.Parameter(torch.randn(8, 8))
    w.mup_width_mult = 4.0
    b = torch.nn.Parameter(torch.randn(8))
    b.mup_width_mult = 4.0
    e = torch.nn.Parameter(torch.randn(3, 8))  # no width multiplier (finite dims)
    return w, b, e


def test_muadam_scales_matrix_like_lr_and_schedules_keep_it():
    w, b, e = _mup_params()
    opt = optim.MuAdam([w, b, e], lr=1e-2, weight_decay=0.1)
    by = {id(p): g for g in opt.param_groups for p in g["params"]}
    assert abs(by[id(w)]["lr"] - 1e-2 / 4) < 1e-12 and abs(by[id(w)]["weight_decay"] - 0.4) < 1e-12
    assert by[id(b)]["lr"] == 1e-2 and by[id(e)]["lr"] == 1e-2
    sched = WarmupLR(opt, warmup_min_lr=0.0, warmup_max_lr=1e-2, warmup_num_steps=2, warmup_type="linear")
    for _ in range(3):
        sched.step()
    assert abs(by[id(w)]["lr"] - 1e-2 / 4) < 1e-12 and abs(by[id(b)]["lr"] - 1e-2) < 1e-12
    cos = WarmupCosineLR(opt, total_num_steps=10, warmup_num_steps=2)
    for _ in range(3):
        cos.step()
    assert abs(by[id(w)]["lr"] * 4 - by[id(b)]["lr"]) < 1e-12
    (w.sum() + b.sum() + e.sum()).backward()
    opt.step()


def test_musgd_vector_and_matrix_rules():
    w, b, e = _mup_params()
    opt = optim.MuSGD([w, b, e], lr=0.1)
    by = {id(p): g for g in opt.param_groups for p in g["params"]}
    assert abs(by[id(w)]["lr"] - 0.1 / 4) < 1e-12 and abs(by[id(b)]["lr"] - 0.4) < 1e-12 and by[id(e)]["lr"] == 0.1


def _engine_muadamw_case(rank, world):
    import shuffle_exchange_amd as sxe
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4))
    model[0].weight.mup_width_mult = 2.0
    cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "MuAdamW", "params": {"lr": 1e-2}},
           "zero_optimization": {"stage": 2},
           "scheduler": {"type": "WarmupLR", "params": {"warmup_min_lr": 0, "warmup_max_lr": 1e-2,
                                                         "warmup_num_steps": 1}}}
    eng, opt, _, _ = sxe.initialize(model=model, config=cfg)
    for _ in range(3):
        loss = eng(torch.randn(2, 16)).pow(2).mean()
        eng.backward(loss)
        eng.step()
    return sorted(g["lr"] for g in eng.optimizer.param_groups)


def test_engine_muadamw_zero2():
    from .dist_utils import run_dist
    lrs = run_dist(_engine_muadamw_case, 1)[0]
    assert abs(lrs[0] * 2 - lrs[-1]) < 1e-9, lrs


def test_contiguous_allocator_defragments_and_repoints_params():
    a = ContiguousMemoryAllocator(100, torch.float32, "cpu")
    t1 = a.allocate_tensor(30)
    t2 = a.allocate_tensor(30)
    t3 = a.allocate_tensor(30)
    t2.fill_(2.0)
    t3.fill_(3.0)
    p = torch.nn.Parameter(torch.empty(0))
    a.assign_to_param(t3, p, 20, (4, 5))
    a.release_tensor(t1)
    assert a.total_free == 40 and a.largest_contiguous == 30
    t4 = a.allocate_tensor(40)  # needs defragmentation
    assert t4.numel() == 40 and a.total_free == 0
    assert torch.all(a.tensor_map[t2._sxe_alloc_id] == 2.0) and torch.all(p == 3.0) and p.shape == (4, 5)
    assert p.data_ptr() == a.buffer.data_ptr() + 30 * 4  # t3 slid down to offset 30
    a.release_tensor(t4)
    assert a.largest_contiguous == 40 and a.max_allocated_memory() == 100


def test_instrument_w_nvtx_is_transparent():
    from shuffle_exchange_amd.utils.nvtx import instrument_w_nvtx

    @instrument_w_nvtx
    def f(x):
        return x + 1
    assert f(1) == 2


def test_zero3_linear_matches_functional():
    from shuffle_exchange_amd.runtime.zero.linear import LinearModuleForZeroStage3, zero3_linear_wrap
    torch.manual_seed(0)
    m = LinearModuleForZeroStage3(8, 4)
    x = torch.randn(3, 8, requires_grad=True)
    y = m(x)
    torch.testing.assert_close(y, torch.nn.functional.linear(x, m.weight, m.bias))
    torch.testing.assert_close(zero3_linear_wrap(x, m.weight, m.bias), y)
    y.sum().backward()
    assert m.weight.grad is not None and x.grad is not None


def test_nhwc_bias_add_variants():
    from shuffle_exchange_amd.ops.spatial import nhwc_bias_add
    x = torch.randn(2, 8, 4, 4).to(memory_format=torch.channels_last)
    o = torch.randn(2, 8, 4, 4).to(memory_format=torch.channels_last)
    b, ob = torch.randn(8), torch.randn(8)
    bb = b.view(1, 8, 1, 1)
    torch.testing.assert_close(nhwc_bias_add(x, b), x + bb)
    torch.testing.assert_close(nhwc_bias_add(x, b, o), x + bb + o)
    torch.testing.assert_close(nhwc_bias_add(x, b, o, ob), x + bb + o + ob.view(1, 8, 1, 1))
    y = torch.randn(2, 4, 4, 8)  # plain NHWC tensor
    torch.testing.assert_close(nhwc_bias_add(y, b), y + b)


def test_loco_error_feedback_bounds_accumulated_quantization_error():
    """LoCo (ops/quantizer.loco_quantize): with error feedback (beta = 1) the sum of the dequantized
    gradients over many steps stays within one quantization step of the true sum, while plain
    quantization accumulates its bias linearly."""
    from shuffle_exchange_amd.ops.quantizer import dequantize, loco_quantize, quantize
    torch.manual_seed(0)
    g = torch.randn(1024) * 1e-3 + 0.37e-3  # constant gradient, biased w.r.t. the int4 grid
    steps, tot_plain, tot_loco, err = 50, torch.zeros(1024), torch.zeros(1024), None
    for _ in range(steps):
        q, s = quantize(g, 128, 4)
        tot_plain += dequantize(q, s, 128, 4, numel=1024, dtype=torch.float32)
        q, s, err = loco_quantize(g, err, 1.0, 128, 4)
        tot_loco += dequantize(q, s, 128, 4, numel=1024, dtype=torch.float32)
    true = g * steps
    e_plain = (tot_plain - true).abs().max().item()
    e_loco = (tot_loco - true).abs().max().item()
    assert e_loco < 0.2 * e_plain, (e_loco, e_plain)


def test_packaged_gemm_table_is_lf_and_has_validators():
    """TunableOp rejects a results file whose lines end in CRLF (the last validator's value then
    carries a carriage return): the packaged MI355X table must be LF-only."""
    import os
    from shuffle_exchange_amd.runtime.gemm_tuning import PACKAGED
    raw = open(PACKAGED, "rb").read()
    assert b"\r" not in raw
    keys = [ln.split(",")[1] for ln in raw.decode().splitlines() if ln.startswith("Validator,")]
    assert {"PT_VERSION", "HIP_VERSION", "HIPBLASLT_VERSION", "GCN_ARCH_NAME", "ROCBLAS_VERSION"} <= set(keys)
    assert os.path.getsize(PACKAGED) > 0


def _comm_api_case(rank, world):
    import torch
    from shuffle_exchange_amd import comm
    outs = [torch.empty(world * 3), torch.empty(world * 2)]
    comm.all_gather_coalesced(outs, [torch.full((3,), float(rank)), torch.full((2,), 10.0 + rank)])
    rs = torch.empty(2)
    comm.reduce_scatter(rs, [torch.ones(2) * (rank + 1), torch.ones(2) * (rank + 1)])
    gl = [torch.empty(1) for _ in range(world)] if rank == 0 else None
    comm.gather(torch.tensor([float(rank)]), gl, dst=0)
    sc = torch.empty(1)
    comm.scatter(sc, [torch.tensor([5.0 + r]) for r in range(world)] if rank == 0 else None, src=0)
    return {"ag": [o.tolist() for o in outs], "rs": rs.tolist(), "gather": [g.item() for g in gl] if gl else None,
            "scatter": sc.item(), "ranks": comm.get_all_ranks_from_group(None), "avail": comm.is_available()}


def test_comm_facade_reference_surface():
    """The rest of the reference comm API (list-form collectives, gather/scatter, discovery) on gloo."""
    from .dist_utils import run_dist
    res = run_dist(_comm_api_case, 2)
    for r, out in enumerate(res):
        assert out["ag"] == [[0.0, 0.0, 0.0, 1.0, 1.0, 1.0], [10.0, 10.0, 11.0, 11.0]]
        assert out["rs"] == [3.0, 3.0]
        assert out["scatter"] == 5.0 + r
        assert out["ranks"] == [0, 1] and out["avail"]
    assert res[0]["gather"] == [0.0, 1.0]
    import shuffle_exchange_amd.comm as c
    ref = ["all_gather_coalesced", "gather", "scatter", "reduce_scatter", "get_all_ranks_from_group",
           "has_all_reduce_coalesced", "has_coalescing_manager", "init_deepspeed_backend", "initialize_mesh_device",
           "mpi_discovery", "set_backend", "timed_op", "in_aml", "in_aws_sm", "in_dlts", "is_available",
           "patch_aml_env_for_torch_nccl_backend", "patch_aws_sm_env_for_torch_nccl_backend",
           "enable_symm_mem_for_group"]
    assert all(hasattr(c, f) for f in ref)
