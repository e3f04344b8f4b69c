"""Mixtral-8x7B training throughput on MI355X (BASELINE.json config "Mixtral 8x7B MoE"): the full
architecture (hidden 4096, 8 experts x FFN 14336, top-2, GQA 32/8, vocab 32000) cut to L decoder
layers so one GPU holds it, ZeRO-3 bf16 AdamW, seq 2048. Reports tokens/s and TFLOP/s counted on
the ACTIVE parameters (2 of 8 experts per token) plus attention. With one GPU the expert-parallel
all-to-all is the identity (ep_size 1); the EP path itself is covered by the multi-process tests.
  python tools/moe_bench.py [--layers 8] [--mbs 2] [--gas 2] [--steps 3]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--mbs", type=int, default=2)
    ap.add_argument("--gas", type=int, default=2)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--ac", action="store_true")
    a = ap.parse_args()
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.models.mixtral import MixtralForCausalLM, mixtral_config
    sxe.init_distributed(verbose=False)
    cfg = mixtral_config("mixtral-8x7b", num_hidden_layers=a.layers, activation_checkpointing=a.ac)
    torch.manual_seed(0)
    with sxe.zero.Init(dtype=torch.bfloat16):
        model = MixtralForCausalLM(cfg)
    ds = {"train_micro_batch_size_per_gpu": a.mbs, "gradient_accumulation_steps": a.gas, "bf16": {"enabled": True},
          "gradient_clipping": 1.0,
          "zero_optimization": {"stage": 3, "stage3_param_persistence_threshold": 100_000,
                                "stage3_max_reuse_distance": 2 * cfg.num_params(),
                                "stage3_max_live_parameters": cfg.num_params()},
          "optimizer": {"type": "AdamW", "params": {"lr": 3e-4, "weight_decay": 0.1}}, "steps_per_print": 10**9}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    gen = torch.Generator(device="cuda").manual_seed(1)

    def step():
        for _ in range(a.gas):
            ids = torch.randint(0, cfg.vocab_size, (a.mbs, a.seq), generator=gen, device="cuda")
            loss = eng(ids, labels=ids)
            eng.backward(loss)
            eng.step()
        return loss

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    tokens = a.mbs * a.gas * a.seq
    d = cfg.hidden_size // cfg.num_attention_heads
    attn_flops = 3 * 2 * 2 * cfg.num_hidden_layers * a.seq * cfg.num_attention_heads * d / 2
    flops_tok = 6 * (cfg.active_params_per_token()) + attn_flops
    print(json.dumps({"model": f"mixtral-8x7b-arch, {a.layers} layers", "params_B": round(cfg.num_params() / 1e9, 2),
                      "active_params_B": round(cfg.active_params_per_token() / 1e9, 2), "seq": a.seq, "mbs": a.mbs,
                      "gas": a.gas, "ms_per_step": round(dt * 1e3, 1), "tokens_per_s": round(tokens / dt, 1),
                      "tflops_active": round(tokens / dt * flops_tok / 1e12, 1),
                      "peak_hbm_GB": round(torch.cuda.max_memory_allocated() / 1e9, 1), "loss": float(loss)}),
          flush=True)


if __name__ == "__main__":
    main()
