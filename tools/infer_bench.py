#!/usr/bin/env python3
"""Serving micro-benchmark of the ragged engine on one MI355X: prefill throughput and steady-state
decode tokens/s for a batch of concurrent sequences (random-init weights, synthetic prompts).

usage: python tools/infer_bench.py [--model llama3-8b] [--batch 64] [--prompt 512] [--gen 64]
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
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--prompt", type=int, default=512)
    ap.add_argument("--gen", type=int, default=64)
    ap.add_argument("--block", type=int, default=64)
    a = ap.parse_args()
    from shuffle_exchange_amd.inference.v2 import RaggedInferenceEngineConfig, build_engine
    from shuffle_exchange_amd.inference.v2.engine_v2 import MemoryConfig, StateManagerConfig
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    over = {"num_hidden_layers": a.layers} if a.layers else {}
    cfg = llama_config(a.model, **over)
    torch.manual_seed(0)
    with torch.device("cuda"):
        model = LlamaForCausalLM(cfg).to(torch.bfloat16)
    sm = StateManagerConfig(max_ragged_batch_size=max(8192, a.batch * a.prompt), max_ragged_sequence_count=a.batch,
                            memory_config=MemoryConfig(fraction=0.6))
    eng = build_engine(model, RaggedInferenceEngineConfig(kv_block_size=a.block, state_manager=sm))
    g = torch.Generator().manual_seed(1)
    prompts = [torch.randint(0, cfg.vocab_size, (a.prompt,), generator=g) for _ in range(a.batch)]
    uids = list(range(a.batch))
    # warm-up (compiles/tunes nothing, but first launches allocate)
    eng.put([10_000], [prompts[0][:128]])
    eng.flush(10_000)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    # prefill in chunks that fit the ragged token budget
    per = max(1, 8192 // a.prompt)
    for i in range(0, a.batch, per):
        lg = eng.put(uids[i:i + per], prompts[i:i + per])
    torch.cuda.synchronize()
    t_prefill = time.perf_counter() - t0
    nxt = [torch.tensor([int(x)]) for x in lg.argmax(-1).tolist()] * 1
    nxt = [torch.tensor([1]) for _ in uids]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.gen):
        lg = eng.put(uids, nxt)
        nxt = [torch.tensor([int(x)]) for x in lg.argmax(-1).tolist()]
    torch.cuda.synchronize()
    t_dec = time.perf_counter() - t0
    out = {"model": a.model, "batch": a.batch, "prompt": a.prompt, "gen": a.gen,
           "prefill_tokens_per_s": round(a.batch * a.prompt / t_prefill, 1),
           "decode_tokens_per_s": round(a.batch * a.gen / t_dec, 1),
           "decode_ms_per_step": round(t_dec / a.gen * 1000, 3),
           "kv_blocks": eng.n_kv_blocks, "free_blocks": eng.free_blocks}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
