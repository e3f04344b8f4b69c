"""Hybrid engine (RLHF loop) on gloo: ZeRO-3 training interleaved with KV-cached generation that
uses the gathered training weights; generation equals greedy decoding with the full model."""
import torch

from .dist_utils import run_dist


def _case(rank, world):
    import shuffle_exchange_amd as sxe
    from ._dist_cases import global_batches, tiny_llama
    model, cfg = tiny_llama(0)
    ds = {"train_micro_batch_size_per_gpu": 2, "hybrid_engine": {"enabled": True, "max_out_tokens": 5},
          "zero_optimization": {"stage": 3, "stage3_param_persistence_threshold": 0},
          "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    prompt = torch.randint(0, cfg.vocab_size, (2, 6), generator=torch.Generator().manual_seed(4))
    outs = []
    for b in global_batches(cfg, world, 2, 16, 2):
        local = b[rank * 2:(rank + 1) * 2]
        loss = eng(local, labels=local)
        eng.backward(loss)
        eng.step()
        outs.append(eng.generate(prompt, max_new_tokens=5))
    # reference greedy decode with the consolidated weights
    sd = eng._zero3_consolidated_16bit_state_dict()
    ref_model, _ = tiny_llama(1)
    ref_model.load_state_dict(sd, strict=False)
    ref_model.eval()
    ids = prompt.clone()
    for _ in range(5):
        with torch.no_grad():
            ids = torch.cat([ids, ref_model(ids)[:, -1].argmax(-1, keepdim=True)], dim=1)
    return {"last": outs[-1], "ref": ids, "type": type(eng).__name__}


def test_hybrid_engine_generate_after_train():
    for r in run_dist(_case, 2):
        assert r["type"] == "SXEHybridEngine"
        assert torch.equal(r["last"].cpu(), r["ref"])


def _case_tp(rank, world, tp):
    import shuffle_exchange_amd as sxe
    from ._dist_cases import global_batches, tiny_llama
    model, cfg = tiny_llama(0)
    ds = {"train_micro_batch_size_per_gpu": 2,
          "hybrid_engine": {"enabled": True, "max_out_tokens": 4, "inference_tp_size": tp},
          "zero_optimization": {"stage": 3, "stage3_param_persistence_threshold": 0},
          "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    prompt = torch.randint(0, cfg.vocab_size, (2, 6), generator=torch.Generator().manual_seed(4))
    outs = []
    for b in global_batches(cfg, 2, 2, 16, 2):
        local = b[rank * 2:(rank + 1) * 2]
        loss = eng(local, labels=local)
        eng.backward(loss)
        eng.step()
        outs.append(eng.generate(prompt))  # shards re-sliced after every step
    return {"outs": [o.cpu() for o in outs], "timing": eng.timing()}


def test_hybrid_engine_inference_tensor_parallel():
    """inference_tp_size = 2 (reference hybrid_engine inference TP): each rank generates from its
    head / FFN / vocab shards of the freshly trained weights; tokens equal the unsharded engine's."""
    tp1 = run_dist(_case_tp, 2, 1)
    tp2 = run_dist(_case_tp, 2, 2)
    for a, b in zip(tp1, tp2):
        for x, y in zip(a["outs"], b["outs"]):
            assert torch.equal(x, y)
        assert b["timing"]["generate_calls"] == 2 and b["timing"]["generated_tokens"] == 16


def test_lora_fuse_matches_unfused():
    from shuffle_exchange_amd.linear.optimized_linear import LoRAConfig, OptimizedLinear
    torch.manual_seed(0)
    lin = OptimizedLinear(32, 48, lora_config=LoRAConfig(lora_r=4, lora_alpha=8), dtype=torch.float32)
    with torch.no_grad():
        lin.lora_weight_2.normal_()
    x = torch.randn(5, 32)
    ref = lin(x)
    lin.fuse_lora()
    fused = lin(x)
    lin.unfuse_lora()
    assert torch.allclose(fused, ref, atol=1e-5) and torch.allclose(lin(x), ref)
