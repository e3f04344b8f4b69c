"""Decode-step latency of the ragged engine on Llama-3-8B (random bf16 weights): eager vs HIP-graph
replay (inference/v2/decode_graphs.py), for several batch sizes at a fixed context.

  python tools/decode_bench.py [--model llama3-8b] [--ctx 1024] [--batches 1,8,32,64] [--steps 32]
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
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--ctx", type=int, default=1024)
    ap.add_argument("--batches", default="1,8,32,64")
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--modes", default="eager,graphs,graphs+fp8",
                    help="comma list of eager | graphs | graphs+<weight_quant> (fp8 W8A16, fp6 / fp4 FP6-LLM "
                         "planes, mxfp8 / mxfp6 / mxfp4 OCP-MX, int8 / int4)")
    a = ap.parse_args()
    from shuffle_exchange_amd.inference.v2 import RaggedInferenceEngineConfig, build_engine
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    cfg = llama_config(a.model)
    torch.manual_seed(0)
    torch.set_default_dtype(torch.bfloat16)
    with torch.device("cuda"):
        model = LlamaForCausalLM(cfg).eval()
    torch.set_default_dtype(torch.float32)
    nparam = sum(p.numel() for p in model.parameters())
    rows = []
    for mode in a.modes.split(","):
        graphs = mode.startswith("graphs")
        eng = build_engine(model, RaggedInferenceEngineConfig(kv_block_size=64, num_kv_blocks=4096,
                                                              decode_graphs=graphs,
                                                              weight_quant=mode.split("+", 1)[1] if "+" in mode else None))
        for B in [int(x) for x in a.batches.split(",")]:
            uids = list(range(B))
            g = torch.Generator().manual_seed(B)
            for u in uids:  # prefill one by one (bounded activation memory)
                eng.put([u], [torch.randint(0, cfg.vocab_size, (a.ctx,), generator=g).tolist()])
            toks = [[1]] * B
            for _ in range(3):  # warm-up (captures the graphs of this bucket)
                eng.put(uids, toks)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                eng.put(uids, toks)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / a.steps * 1e3
            hbm_gb = (nparam * 2 + B * (a.ctx + a.steps) * cfg.num_hidden_layers * 2 * cfg.num_key_value_heads *
                      (cfg.hidden_size // cfg.num_attention_heads) * 2) / 1e9
            rows.append({"mode": mode, "batch": B, "ctx": a.ctx, "ms_per_step": round(ms, 3),
                         "tokens_per_s": round(B / ms * 1e3, 1), "hbm_GB_per_step": round(hbm_gb, 2),
                         "eff_TB_per_s": round(hbm_gb / ms, 2)})
            print(json.dumps(rows[-1]), flush=True)
            for u in uids:
                eng.flush(u)
        del eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
