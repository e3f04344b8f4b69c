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
