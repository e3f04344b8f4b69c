#!/usr/bin/env python3
"""Headline benchmark: Llama-3-8B, ZeRO-3, bf16, tokens/s on N MI355X GPUs (one process per GPU).

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1 launched by
``torch.distributed.run`` (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* from env, RCCL backend). W untimed
steps, then EXACTLY K timed optimizer steps bracketed by barrier + device sync; the time is the MAX
over ranks; rank 0 prints one JSON line. Every timed step is a full training step: forward, backward,
gradient reduce-scatter, fused AdamW on fp32 masters (all 8.03B parameters), no skipped work.
Data: synthetic token ids (uniform over the 128256-token vocabulary); weights: random init of the
exact Llama-3-8B architecture (no network access for checkpoints/datasets).
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--seq", type=int, default=int(os.environ.get("SXE_BENCH_SEQ", 2048)))
    # global batch 16 per GPU as 8 x 2 micro-steps: 288 GB HBM holds the activations of 8 x 2048
    # tokens (peak 211 GB); half the weight-gradient accumulation passes of 4 x 4 and larger GEMM M
    # (measured 24,254 vs 23,799 tok/s, profiles/bench_1gpu_r02.log)
    ap.add_argument("--mbs", type=int, default=int(os.environ.get("SXE_BENCH_MBS", 8)))
    ap.add_argument("--gas", type=int, default=int(os.environ.get("SXE_BENCH_GAS", 2)))
    ap.add_argument("--stage", type=int, default=3)
    ap.add_argument("--ac", action="store_true", help="activation checkpointing")
    ap.add_argument("--layers", type=int, default=None, help="override layer count (debug only; invalid for the metric)")
    ap.add_argument("--profile-steps", type=int, default=0)
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu = plumbing dry-run over gloo (tests only; invalid for the metric)")
    args = ap.parse_args()
    on_gpu = args.device == "cuda"

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd import comm as dist
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config

    dist.init_distributed(verbose=False)
    world = dist.get_world_size()
    rank = dist.get_rank()
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.manual_seed(1234)
    over = {"activation_checkpointing": args.ac, "max_position_embeddings": max(8192, args.seq)}
    if args.layers:
        over["num_hidden_layers"] = args.layers
    cfg = llama_config(args.model, **over)
    dev = torch.device("cuda", torch.cuda.current_device()) if on_gpu else torch.device("cpu")
    with sxe.zero.Init(dtype=torch.bfloat16):
        model = LlamaForCausalLM(cfg)
    ds_config = {
        "train_micro_batch_size_per_gpu": args.mbs,
        "gradient_accumulation_steps": args.gas,
        "bf16": {"enabled": True},
        "gradient_clipping": 1.0,
        "zero_optimization": {"stage": args.stage, "overlap_comm": True, "reduce_bucket_size": 500_000_000,
                              "stage3_param_persistence_threshold": 100_000, "prefetch_depth": 2,
                              # 288 GB HBM: the whole bf16 model (16 GB for 8B) may stay gathered from
                              # its forward use to its backward re-use -> no backward all-gather
                              "stage3_max_reuse_distance": 2 * cfg.num_params(),
                              "stage3_max_live_parameters": cfg.num_params(),
                              # and keep fp32 gradient sums local across the grad-accumulation
                              # micro-steps: one reduce-scatter per step instead of one per micro-step
                              "stage3_defer_reduce": True,
                              # gathered weights stay valid until the optimizer step: gather once per step
                              "stage3_retain_params_in_step": True},
        "optimizer": {"type": "AdamW", "params": {"lr": 3e-4, "betas": [0.9, 0.95], "eps": 1e-8,
                                                   "weight_decay": 0.1}},
        "steps_per_print": 1000000,
    }
    engine, _, _, _ = sxe.initialize(model=model, config=ds_config)
    n_params = sum(p.numel() for p in model.parameters())
    gen = torch.Generator(device=dev)
    gen.manual_seed(1000 + rank)

    def train_step():
        for i in range(args.gas):
            # a fresh synthetic batch every micro-step (generated on the device: no H2D in the loop)
            batch = torch.randint(0, cfg.vocab_size, (args.mbs, args.seq), generator=gen, device=dev)
            loss = engine(batch, labels=batch)
            engine.backward(loss)
            engine.step()
        return loss

    for _ in range(args.warmup):
        loss = train_step()
    sync()
    dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = train_step()
    sync()
    dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    tokens = args.gpus * args.mbs * args.gas * args.seq * args.steps
    tps = tokens / elapsed
    flops_tok = cfg.flops_per_token(args.seq)
    mfu_tflops = tps * flops_tok / args.gpus / 1e12
    valid = (args.layers is None and args.model == "llama3-8b" and args.stage == 3 and on_gpu and args.seq == 2048
             and args.mbs * args.gas == 16)
    if rank == 0:
        out = {
            "metric": "tokens/sec Llama-3-8B ZeRO-3 bf16 (training, whole job)",
            "value": round(tps, 2),
            "unit": "tokens/s",
            "n_gpus": args.gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1000.0, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic",
            "config": {"model": args.model, "global_batch": args.gpus * args.mbs * args.gas, "seq_len": args.seq,
                       "micro_batch_per_gpu": args.mbs, "grad_accum": args.gas,
                       "parallelism": f"zero{args.stage}-dp{args.gpus}", "params": n_params,
                       "activation_checkpointing": args.ac, "optimizer": "AdamW(fp32 master, fused HIP)"},
            "tflops_per_gpu": round(mfu_tflops, 1),
            "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2**30, 1) if on_gpu else None,
            "final_loss": round(float(loss.detach()), 4),
            "valid_for_metric": valid,
        }
        print(json.dumps(out), flush=True)
    dist.barrier()
    if dist.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
