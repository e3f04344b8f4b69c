"""Mixtral-style MoE training through the engine on the MI355X (ZeRO-3 bf16, TunableOp GEMM table
loaded, top-2 routing with capacity, per-expert GEMMs + HIP SwiGLU): losses finite and falling,
ZeRO-3 parameters stay finite."""
import pytest
import torch

from .dist_utils import run_dist

pytestmark = pytest.mark.gpu


def _case(rank, world, stage):
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.models import MixtralForCausalLM, mixtral_config
    torch.cuda.set_device(0)
    torch.manual_seed(0)
    cfg = mixtral_config("mixtral-tiny", hidden_size=512, intermediate_size=1024, num_attention_heads=4,
                         num_key_value_heads=2, vocab_size=2048, num_hidden_layers=2, num_local_experts=8)
    with sxe.zero.Init(dtype=torch.bfloat16):
        model = MixtralForCausalLM(cfg)
    ds = {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": 1, "bf16": {"enabled": True},
          "zero_optimization": {"stage": stage}, "gradient_clipping": 1.0,
          "optimizer": {"type": "AdamW", "params": {"lr": 3e-3}}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    ids = torch.randint(0, 2048, (2, 256), generator=torch.Generator().manual_seed(1)).cuda()
    losses = []
    for _ in range(6):
        loss = eng(ids, labels=ids)
        eng.backward(loss)
        eng.step()
        losses.append(float(loss))
    torch.cuda.synchronize()
    return losses


@pytest.mark.parametrize("stage", [2, 3])
def test_moe_engine_trains_on_gpu(stage):
    losses = run_dist(_case, 1, stage)[0]
    assert all(l == l and l < 1e4 for l in losses), losses
    assert losses[-1] < losses[0], losses


@pytest.fixture
def _hip():
    from shuffle_exchange_amd.ops import native
    native.require_hip()


@pytest.mark.parametrize("E,k", [(8, 2), (64, 1), (160, 6), (512, 2)])
def test_topk_softmax_kernel_vs_torch(_hip, E, k):
    """moe.hip fused softmax + top-k == torch softmax / topk; softmax backward == autograd of torch."""
    from shuffle_exchange_amd.ops.moe import topk_softmax
    g = torch.Generator(device="cuda").manual_seed(E)
    logits = torch.randn(1000, E, device="cuda", generator=g).requires_grad_()
    probs, idx = topk_softmax(logits, k)
    ref = torch.softmax(logits.detach().float(), -1)
    assert torch.allclose(probs, ref, atol=1e-6)
    assert torch.equal(idx, torch.topk(logits.detach(), k, dim=1).indices)
    gp = torch.randn_like(probs)
    (probs * gp).sum().backward()
    l2 = logits.detach().clone().requires_grad_()
    (torch.softmax(l2, -1) * gp).sum().backward()
    assert torch.allclose(logits.grad, l2.grad, atol=1e-6)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_dispatch_combine_kernels_vs_torch(_hip, dtype):
    """moe.hip dispatch / combine (and both backwards) == the PyTorch reference path, with dropped
    assignments and empty capacity slots."""
    from shuffle_exchange_amd.ops import moe as M
    torch.manual_seed(0)
    S, H, E, C, k = 300, 256, 8, 48, 2
    expert = torch.randint(0, E, (S, k), device="cuda")
    loc = torch.randint(0, C, (S, k), device="cuda")
    # make (expert, loc) unique per kept assignment and drop ~10 %
    flat = expert * C + loc
    first = torch.zeros(E * C, dtype=torch.bool, device="cuda")
    keep = torch.zeros(S * k, dtype=torch.bool, device="cuda")
    for i, f in enumerate(flat.reshape(-1).tolist()):
        if not first[f] and (i % 10):
            first[f] = True
            keep[i] = True
    keep = keep.view(S, k)
    slots, slot_src = M.routing_tables(expert, loc, keep, C, E)
    x = torch.randn(S, H, device="cuda", dtype=dtype, requires_grad=True)
    w = torch.rand(S, k, device="cuda", requires_grad=True)
    out_rows = torch.randn(E * C, H, device="cuda", dtype=dtype, requires_grad=True)

    d = M.dispatch(x, slots, slot_src)
    y = M.combine(out_rows, slots, slot_src, w)
    gd, gy = torch.randn_like(d), torch.randn_like(y)
    (d.float() * gd.float()).sum().backward()
    (y.float() * gy.float()).sum().backward()

    xr, wr, orr = (t.detach().float().cpu().requires_grad_() for t in (x, w, out_rows))
    sc, ssc = slots.cpu(), slot_src.cpu()
    dr = M.dispatch(xr, sc, ssc)
    yr = M.combine(orr, sc, ssc, wr)
    (dr * gd.float().cpu()).sum().backward()
    (yr * gy.float().cpu()).sum().backward()
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    assert torch.allclose(d.float().cpu(), dr, atol=tol)
    assert torch.allclose(y.float().cpu(), yr, atol=tol, rtol=tol)
    assert torch.allclose(x.grad.float().cpu(), xr.grad, atol=tol, rtol=tol)
    assert torch.allclose(out_rows.grad.float().cpu(), orr.grad, atol=tol, rtol=tol)
    assert torch.allclose(w.grad.cpu(), wr.grad, atol=tol * 10, rtol=tol)


def test_moe_layer_gpu_kernels_match_cpu_path(_hip):
    """The MoE layer on the GPU (HIP gating / dispatch / combine) == the same layer on the CPU path."""
    import copy
    from shuffle_exchange_amd.moe.layer import MoE
    torch.manual_seed(0)
    expert = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.GELU(), torch.nn.Linear(128, 64))
    layer = MoE(64, expert, num_experts=4, k=2, capacity_factor=1.5, min_capacity=4, top2_2nd_expert_sampling=False)
    gpu = copy.deepcopy(layer).cuda()
    x = torch.randn(2, 50, 64)
    yc = layer(x)[0]
    yg = gpu(x.cuda())[0]
    assert torch.allclose(yg.cpu(), yc, atol=1e-4), (yg.cpu() - yc).abs().max()
    yc.sum().backward()
    yg.sum().backward()
    for (n, a), (_, b) in zip(layer.named_parameters(), gpu.named_parameters()):
        assert torch.allclose(b.grad.cpu(), a.grad, atol=1e-4), n
