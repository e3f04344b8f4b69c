"""Per-step losses of the eager and the FX-compiled engine on a cut full-width Llama-3-8B (same
batch every step), to locate where a compiled trajectory departs from the eager one.
  python tools/compile_parity_probe.py [--layers 1] [--stage 1] [--steps 4] [--seq 512] [--mbs 2]
"""
import argparse
import gc
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(compiled, a):
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    cfg = llama_config("llama3-8b", num_hidden_layers=a.layers)
    torch.manual_seed(0)
    model = LlamaForCausalLM(cfg).to(device="cuda", dtype=torch.bfloat16)
    ds = {"train_micro_batch_size_per_gpu": a.mbs, "bf16": {"enabled": True},
          "optimizer": {"type": "AdamW", "params": {"lr": a.lr}},
          "zero_optimization": {"stage": a.stage}, "compile": {"deepcompile": True, "fx_zero3": True}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    if compiled:
        eng.compile()
    g = torch.Generator(device="cuda").manual_seed(1)
    ids = torch.randint(0, cfg.vocab_size, (a.mbs, a.seq), device="cuda", generator=g)
    losses, gnorms = [], []
    for _ in range(a.steps):
        loss = eng(ids, labels=ids)
        eng.backward(loss)
        eng.step()
        losses.append(round(float(loss.detach()), 5))
        gn = eng.get_global_grad_norm()
        gnorms.append(None if gn is None else round(float(gn), 4))
    del eng, model
    gc.collect()
    torch.cuda.empty_cache()
    torch._dynamo.reset()
    return {"compiled": compiled, "losses": losses, "grad_norms": gnorms}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=1)
    ap.add_argument("--stage", type=int, default=1)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--mbs", type=int, default=2)
    ap.add_argument("--lr", type=float, default=1e-5)
    a = ap.parse_args()
    import shuffle_exchange_amd as sxe
    sxe.init_distributed(verbose=False)
    env = {k: v for k, v in os.environ.items() if k.startswith("SXE_")}
    for c in (False, True):
        out = run(c, a)
        out["env"] = env
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
