"""DeepCompile on MI355X: compiled (FX graph compiler, compile/fx_backend.py and compile/fx_zero3.py)
vs eager step time of a cut Llama-3-8B (full width, L layers) under ZeRO-1 / 2 / 3, bf16 AdamW.

One GPU: the partition group has one rank, so ZeRO-3's gathers are local (every unit persistent)
and the comparison measures what the graph compiler changes on the device -- the Dynamo / AOT
graph executed as generated Python over the same HIP kernels, gradients handed to the optimizer
by in-graph reduce nodes -- against the eager engine with its autograd hooks. The ZeRO-3
gather / release / prefetch placement itself is pinned by the gloo tests
(tests/test_compile_fx.py).
  python tools/compile_bench.py [--layers 4] [--seq 2048] [--mbs 2] [--stages 1,2,3] [--steps 5] [--offload-param]
                                [--only eager|compiled]
"""
import argparse
import gc
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(stage, compiled, a):
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    cfg = llama_config("llama3-8b", num_hidden_layers=a.layers)
    torch.manual_seed(0)
    model = LlamaForCausalLM(cfg).to(device="cuda", dtype=torch.bfloat16)
    z = {"stage": stage, "reduce_bucket_size": 500_000_000}
    if stage == 3 and a.offload_param:
        # parameters on the host: even one GPU gathers every unit (H2D) per use, which is where the
        # graph compiler's in-graph prefetch / release placement can show up
        z.update({"offload_param": {"device": "cpu", "pin_memory": True}, "stage3_param_persistence_threshold": 0})
    ds = {"train_micro_batch_size_per_gpu": a.mbs, "bf16": {"enabled": True},
          "optimizer": {"type": "AdamW", "params": {"lr": 1e-5}},
          "zero_optimization": z, "compile": {"deepcompile": True, "fx_zero3": True}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    from torch._dynamo.utils import counters
    counters.clear()
    if compiled:
        eng.compile()
    g = torch.Generator(device="cuda").manual_seed(1)
    ids = torch.randint(0, cfg.vocab_size, (a.mbs, a.seq), device="cuda", generator=g)

    def step():
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
    ms = (time.perf_counter() - t0) * 1e3 / a.steps
    out = {"stage": stage, "offload_param": bool(stage == 3 and a.offload_param), "compiled": compiled,
           "ms_per_step": round(ms, 2),
           "tokens_per_s": round(a.mbs * a.seq * 1e3 / ms, 1), "loss": round(float(loss.detach()), 4)}
    if compiled:
        fx = eng.compile_plan["fx"]
        out["graph_reduces"] = sum(v.get("reduces", 0) for v in fx.graphs.values())
        out["graphs"] = len(fx.graphs)
        out["graph_breaks"] = sum(counters["graph_break"].values())
    del eng, model
    gc.collect()
    torch.cuda.empty_cache()
    torch._dynamo.reset()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--mbs", type=int, default=2)
    ap.add_argument("--stages", default="1,2,3")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--offload-param", action="store_true", help="ZeRO-3 with offload_param cpu")
    ap.add_argument("--only", choices=["eager", "compiled"], default=None,
                    help="run one arm (per-arm kernel traces)")
    a = ap.parse_args()
    import shuffle_exchange_amd as sxe
    sxe.init_distributed(verbose=False)
    for s in (int(x) for x in a.stages.split(",")):
        if a.only:
            print(json.dumps(run(s, a.only == "compiled", a)), flush=True)
            continue
        e = run(s, False, a)
        print(json.dumps(e), flush=True)
        c = run(s, True, a)
        c["speedup_vs_eager"] = round(e["ms_per_step"] / c["ms_per_step"], 3)
        print(json.dumps(c), flush=True)


if __name__ == "__main__":
    main()
