#!/usr/bin/env python3
"""Training benchmarks on N MI355X GPUs (one process per GPU, RCCL over xGMI), one per BASELINE.json config.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1 launched by
``torch.distributed.run`` (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* from env). W untimed steps, then
EXACTLY K timed optimizer steps bracketed by barrier + device sync; the time is the MAX over ranks;
rank 0 prints one JSON line. Every timed step is a full training step: forward, backward, gradient
reduction, optimizer step on fp32 masters for every parameter -- no skipped work.
Data: synthetic token ids (uniform over the vocabulary); weights: random init of the named
architecture (no network access for checkpoints/datasets).

``--config`` (default ``llama8b-z3``, the headline):
  llama8b-z3          Llama-3-8B, ZeRO-3, bf16, seq 2048, 16 sequences per GPU (8 x 2 micro-steps),
                      MI355X-tuned residency (288 GB HBM: gathered weights kept for the step,
                      gradient sums reduce-scattered once per step) -- BASELINE.json metric
  llama8b-z3-default  the same model/batch with the REFERENCE's default ZeRO-3 knobs (a gather per
                      micro-step forward, backward re-gathers beyond reuse distance 1e9 / max_live
                      1e9, a reduce-scatter every micro-step, prefetch bucket 5e7)
  mixtral-ep          Mixtral-8x7B, expert parallel over all N GPUs (ep = N, one all-to-all pair per
                      MoE layer), ZeRO-2 (the reference asserts MoE off at stage 3, engine.py:1760),
                      seq 2048; min(32, 8N) layers so the experts per GPU stay fixed (full 32 at N >= 4)
  llama70b-infinity   Llama-3-70B, ZeRO-3 + ZeRO-Infinity optimizer offload to pinned host DRAM
                      (C++ AVX-512 Adam), activation checkpointing by HBM budget (auto_ac_policy:
                      none while 10N layers' activations fit), seq 2048; 10N layers up to the
                      full 80 (host DRAM of one node bounds the fp32 state: 12 B/param)
  llama8b-sp32k       Llama-3-8B, Ulysses sequence parallel over all N GPUs, seq 32768, ZeRO-3; one 32k
                      sequence per SP group (strong scaling); activation checkpointing by HBM budget
                      (auto_ac_policy: none when the activations fit -- from 2 GPUs --, else the
                      MLP-only policy that keeps the attention outputs, else full layers)
Every JSON line carries the full ZeRO/SP/EP configuration, the measured per-step communication
volume per collective (``comm_measured``: calls and bytes per rank per step, from the comm facade's
counters) and an analytic model of it (``comm_model``), so a scaling curve can be checked against the
bytes that crossed xGMI.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

CONFIGS = {
    "llama8b-z3": dict(family="llama", model="llama3-8b", seq=2048, mbs=8, gas=2, stage=3, knobs="tuned",
                       metric="tokens/sec Llama-3-8B ZeRO-3 bf16 (training, whole job)"),
    "llama8b-z3-default": dict(family="llama", model="llama3-8b", seq=2048, mbs=8, gas=2, stage=3, knobs="reference",
                               metric="tokens/sec Llama-3-8B ZeRO-3 bf16 (training, whole job)"),
    "mixtral-ep": dict(family="mixtral", model="mixtral-8x7b", seq=2048, mbs=2, gas=2, stage=2, knobs="tuned",
                       ep=True, metric="tokens/sec Mixtral-8x7B expert-parallel bf16 (training, whole job)"),
    "llama70b-infinity": dict(family="llama", model="llama3-70b", seq=2048, mbs=2, gas=2, stage=3, knobs="reference",
                              offload=True, ac=True, ac_policy="auto",
                              metric="tokens/sec Llama-3-70B ZeRO-3 + ZeRO-Infinity host offload bf16 "
                                     "(training, whole job)"),
    "llama8b-sp32k": dict(family="llama", model="llama3-8b", seq=32768, mbs=1, gas=1, stage=3, knobs="tuned", sp=True,
                          ac=True, ac_policy="auto", metric="tokens/sec Llama-3-8B Ulysses SP seq 32k bf16 (training, whole job)"),
}


def default_layers(name, world):
    """Layer count of the model for a config at `world` GPUs (None = the full architecture)."""
    if name == "mixtral-ep":
        return None if world >= 4 else 8 * world
    if name == "llama70b-infinity":
        return None if world >= 8 else 10 * world
    return None


def zero_knobs(c, cfg, stage):
    z = {"stage": stage, "overlap_comm": True, "reduce_bucket_size": 500_000_000}
    if stage == 3:
        z.update({"stage3_param_persistence_threshold": 100_000})
        if c["knobs"] == "tuned":
            z.update({"prefetch_depth": 2,
                      # 288 GB HBM: the whole bf16 model (16 GB for 8B) may stay gathered from its
                      # forward use to its backward re-use -> no backward all-gather
                      "stage3_max_reuse_distance": 2 * cfg.num_params(),
                      "stage3_max_live_parameters": cfg.num_params(),
                      # fp32 gradient sums stay local across the micro-steps: one reduce-scatter per step
                      "stage3_defer_reduce": True,
                      # gathered weights stay valid until the optimizer step: gather once per step
                      "stage3_retain_params_in_step": True})
        else:  # the reference's defaults (runtime/zero/config.py)
            z.update({"stage3_prefetch_bucket_size": 50_000_000, "stage3_max_live_parameters": 1_000_000_000,
                      "stage3_max_reuse_distance": 1_000_000_000})
    if c.get("offload"):
        z["offload_optimizer"] = {"device": "cpu", "pin_memory": True}
    return z


# Saved activation bytes per token per Llama decoder layer (bf16, fused kernels of this repo) with
# no checkpointing / with only the MLP sub-block checkpointed, at hidden 4096 / FFN 14336: the MLP
# keeps gate_up (2 x 14336), the SwiGLU output and its token-minor copy for the weight gradients.
ACT_BYTES_PER_TOKEN_LAYER = {"none": 170e3, "mlp": 55e3}


def auto_ac_policy(model_name, layers, tokens_per_gpu, world, stage, hbm_bytes=288e9, budget=0.75,
                   partial_budget=0.90, state_bytes=16.0):
    """The least recompute that fits, as (policy, checkpointed layers or None = all): no
    checkpointing if the saved activations and the ZeRO states fit `budget` of HBM; else the MLP-only
    policy (attention outputs kept: the flash forward is not re-run) on as FEW layers as keep the
    modelled bytes within `partial_budget` (the other layers keep their MLP activations: 288 GB holds
    part of them -- at Llama-3-8B 32k tokens on one GPU, MLP recompute in every layer peaks at 204 GB
    measured, ~18 GB above this model, and each layer left whole adds 2.6 GB measured vs 3.8 modelled:
    21 checkpointed layers peaked at 234 GB, 15 at 249 GB, profiles/r06/sp32k/); else full-layer
    checkpointing. 288 GB per MI355X makes
    'none' the answer for Llama-3-8B at 32k tokens from 2 GPUs up."""
    from shuffle_exchange_amd.models import llama_config
    cfg = llama_config(model_name, **({"num_hidden_layers": layers} if layers else {}))
    # HBM bytes per parameter of the ZeRO states: 16 (bf16 param, fp32 grad, master, moments), 6 with
    # the optimizer offloaded to the host (bf16 param + fp32 gradient accumulator)
    states = state_bytes * cfg.num_params() / (world if stage == 3 else 1)
    scale = (cfg.hidden_size / 4096 + cfg.intermediate_size / 14336) / 2
    L = cfg.num_hidden_layers
    per = {k: v * scale * tokens_per_gpu for k, v in ACT_BYTES_PER_TOKEN_LAYER.items()}
    if states + per["none"] * L <= budget * hbm_bytes:
        return "none", None
    if states + per["mlp"] * L <= budget * hbm_bytes:
        for n in range(L + 1):  # fewest MLP-checkpointed layers within the partial budget
            if states + per["mlp"] * n + per["none"] * (L - n) <= partial_budget * hbm_bytes:
                return ("none", None) if n == 0 else ("mlp", None if n == L else n)
        return "mlp", None
    return "full", None


def comm_model(opt, world, stage, knobs, gas, elem_bytes=2):
    """Analytic per-rank payload bytes per optimizer step of the ZeRO collectives (rccl-tests payload
    convention: gathered size for all-gather, input size for reduce-scatter / all-reduce)."""
    if world == 1 or opt is None:
        return {}
    out = {}
    if stage == 3 and hasattr(opt, "fgroups"):
        S = opt.S
        if S == 1:
            return {}
        # the gather policy of runtime/zero/stage3.py replayed on the recorded forward trace
        size = {fg.idx: sum(u.padded for u in fg.units if not u.persistent) for fg in opt.fgroups}
        # frozen units are gathered but never reduced, nor refreshed after the step
        rs_size = sum(u.padded for fg in opt.fgroups for u in fg.units
                      if not u.persistent and not getattr(u, "frozen", False))
        persistent = sum(u.padded for fg in opt.fgroups for u in fg.units
                         if u.persistent and not getattr(u, "frozen", False))
        trace = list(opt.trace)
        if getattr(opt, "retain_params", False):
            gathered = sum(size[i] for i in trace)  # once per step: retained until the boundary backward
        else:
            dist_, kept, live = opt._reuse_distances(), set(), 0
            for i in trace:  # _keep_for_backward, in forward order
                if i == trace[-1]:
                    kept.add(i)
                elif (opt.max_reuse_distance > 0 and dist_.get(i, 1 << 62) < opt.max_reuse_distance
                      and live + size[i] <= opt.max_live_parameters):
                    kept.add(i)
                    live += size[i]
            gathered = gas * (sum(size[i] for i in trace) + sum(size[i] for i in trace if i not in kept))
        n_rs = 1 if getattr(opt, "defer_reduce", False) else gas
        out["all_gather_into_tensor"] = (gathered + persistent) * elem_bytes  # persistent: refreshed after the step
        out["reduce_scatter_tensor"] = n_rs * (rs_size + persistent) * elem_bytes
    elif stage in (1, 2) and hasattr(opt, "units"):
        total = sum(u.padded for units in opt.units for u in units if u.topo.S > 1) * elem_bytes
        out["reduce_scatter_tensor"] = total * (gas if stage == 2 else 1)
        out["all_gather_into_tensor"] = total
    return out


def effective_zero(opt):
    """The ZeRO behaviour the run actually had (config knobs can be inert: e.g. the deferred reduce
    and the retained gathers need a partition group of more than one rank)."""
    if opt is None:
        return {}
    if hasattr(opt, "fgroups"):  # stage 3
        units = [u for us in opt.units for u in us]
        return {"partition_size": opt.S, "defer_reduce": bool(opt.defer_reduce),
                "retain_params_in_step": bool(opt.retain_params), "prefetch_depth": opt.prefetch_depth,
                "prefetch_numel": opt.prefetch_numel, "max_reuse_distance": opt.max_reuse_distance,
                "max_live_parameters": opt.max_live_parameters, "units": len(units),
                "persistent_units": sum(1 for u in units if u.persistent),
                "reduce_communicator_separate": opt.reduce_group is not None
                and opt.reduce_group is not opt.topo.slice_group}
    if hasattr(opt, "units") and hasattr(opt, "topo"):  # stage 1/2
        return {"stage": getattr(opt, "stage", None), "partition_size": opt.topo.S,
                "units": sum(len(us) for us in opt.units),
                "shuffle_exchange": getattr(opt, "shuffle_exchange_enabled", False)}
    return {"optimizer": type(opt).__name__}


def _attribute_step(train_step, out_dir):
    """Profile one step with torch.profiler and write, per GPU kernel, the op and Python call sites
    that launched it (what a rocprofv3 kernel table cannot say): ``attrib_kernels.txt``."""
    from torch.profiler import ProfilerActivity, profile
    os.makedirs(out_dir, exist_ok=True)
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        train_step()
        torch.cuda.synchronize()
    with open(os.path.join(out_dir, "attrib_ops.txt"), "w") as f:
        f.write(prof.key_averages(group_by_stack_n=6).table(sort_by="self_cuda_time_total", row_limit=80,
                                                             max_name_column_width=90, max_src_column_width=200))
    ev = [e for e in prof.events() if e.device_type.name == "CUDA"] if hasattr(prof, "events") else []
    agg = {}
    for e in ev:
        p = e.cpu_parent
        chain = []
        while p is not None and len(chain) < 4:
            chain.append(p.name)
            p = p.cpu_parent
        stack = [s for s in (getattr(e.cpu_parent, "stack", None) or []) if "shuffle_exchange_amd" in s or "bench.py" in s]
        key = (e.name[:90], " < ".join(chain), " | ".join(stack[:3]))
        a = agg.setdefault(key, [0, 0.0])
        a[0] += 1
        a[1] += e.device_time_total / 1000.0 if hasattr(e, "device_time_total") else e.cuda_time_total / 1000.0
    with open(os.path.join(out_dir, "attrib_kernels.txt"), "w") as f:
        for (k, chain, stack), (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:120]:
            f.write(f"{ms:9.2f} ms {n:5d}x  {k}\n      ops: {chain}\n      at: {stack}\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default=os.environ.get("SXE_BENCH_CONFIG", "llama8b-z3"), choices=sorted(CONFIGS))
    ap.add_argument("--model", default=None, help="override the architecture preset (tests: llama-tiny / mixtral-tiny)")
    ap.add_argument("--seq", type=int, default=None)
    ap.add_argument("--mbs", type=int, default=None)
    ap.add_argument("--gas", type=int, default=None)
    ap.add_argument("--stage", type=int, default=None)
    ap.add_argument("--ac", action="store_true", help="activation checkpointing")
    ap.add_argument("--ac-policy", default=None, choices=["full", "mlp", "none", "auto"],
                    help="what activation checkpointing recomputes (default: the config's; auto = the "
                         "least recompute whose saved activations fit the HBM budget)")
    ap.add_argument("--ac-layers", type=int, default=None,
                    help="checkpoint only the first N decoder layers (default: all, or auto's choice)")
    ap.add_argument("--layers", type=int, default=None, help="override layer count (a cut model: not the metric)")
    ap.add_argument("--offload-ratio", type=float, default=None,
                    help="offload configs: Twin-Flow offload_optimizer.ratio (share of the optimizer on the "
                         "host; default 1.0 = the whole optimizer, the reference's ZeRO-Infinity setting)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu = plumbing dry-run over gloo (tests only; invalid for the metric)")
    args = ap.parse_args()
    c = CONFIGS[args.config]
    on_gpu = args.device == "cuda"
    seq = args.seq or int(os.environ.get("SXE_BENCH_SEQ", c["seq"]))
    # llama8b-z3: 16 sequences per GPU as 8 x 2 micro-steps -- 288 GB HBM holds the activations of
    # 8 x 2048 tokens (peak 211 GB); half the weight-gradient accumulation passes of 4 x 4
    mbs = args.mbs or int(os.environ.get("SXE_BENCH_MBS", c["mbs"]))
    gas = args.gas or int(os.environ.get("SXE_BENCH_GAS", c["gas"]))
    stage = c["stage"] if args.stage is None else args.stage
    model_name = args.model or c["model"]

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd import comm as dist

    dist.init_distributed(verbose=False)
    world = dist.get_world_size()
    rank = dist.get_rank()
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    sp = world if c.get("sp") else 1
    ep = world if c.get("ep") else 1
    dp = world // sp
    layers = args.layers if args.layers is not None else default_layers(args.config, world)
    ac = args.ac or bool(c.get("ac"))
    policy = args.ac_policy or c.get("ac_policy") or ("full" if ac else "none")
    ac_layers = None
    if policy == "auto":
        policy, ac_layers = auto_ac_policy(model_name, layers, seq // sp * mbs, world, stage,
                                           state_bytes=6.0 if c.get("offload") else 16.0)
    if args.ac_layers is not None:
        ac_layers = args.ac_layers
    ac = policy != "none"
    torch.manual_seed(1234)
    over = {"activation_checkpointing": ac, "max_position_embeddings": max(8192, seq)}
    if c["family"] == "llama" and policy == "mlp":
        over["ac_policy"] = "mlp"
    if ac and ac_layers is not None:
        over["ac_layers"] = ac_layers
    if layers:
        over["num_hidden_layers"] = layers
    if sp > 1:
        over["sequence_parallel"] = True
    if c["family"] == "mixtral":
        from shuffle_exchange_amd.models.mixtral import MixtralForCausalLM, mixtral_config
        if ep > 1:
            over["ep_size"] = ep
        cfg = mixtral_config(model_name, **over)
        ctor = MixtralForCausalLM
    else:
        from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
        cfg = llama_config(model_name, **over)
        ctor = LlamaForCausalLM
    dev = torch.device("cuda", torch.cuda.current_device()) if on_gpu else torch.device("cpu")
    if stage == 3:
        with sxe.zero.Init(dtype=torch.bfloat16):
            model = ctor(cfg)
    else:
        model = ctor(cfg)
    zero = zero_knobs(c, cfg, stage)
    if args.offload_ratio is not None and "offload_optimizer" in zero:
        zero["offload_optimizer"]["ratio"] = float(args.offload_ratio)
    ds_config = {
        "train_micro_batch_size_per_gpu": mbs,
        "gradient_accumulation_steps": gas,
        "bf16": {"enabled": True},
        "gradient_clipping": 1.0,
        "zero_optimization": zero,
        "optimizer": {"type": "AdamW", "params": {"lr": 3e-4, "betas": [0.9, 0.95], "eps": 1e-8,
                                                   "weight_decay": 0.1}},
        "steps_per_print": 1000000,
    }
    if sp > 1:
        ds_config["sequence_parallel_size"] = sp
    engine, _, _, _ = sxe.initialize(model=model, config=ds_config)
    n_params = sum(getattr(p, "ds_numel", p.numel()) for p in model.parameters())
    if c.get("ep"):
        n_params = cfg.num_params()  # every expert of the architecture (each rank holds 1/ep of them)
    gen = torch.Generator(device=dev)
    # one data stream per data-parallel replica; the ranks of an SP group shard the same sequences
    gen.manual_seed(1000 + rank // sp)
    from shuffle_exchange_amd.parallel import groups
    sp_rank = groups.get_sequence_parallel_rank() if sp > 1 else 0

    def train_step():
        for _ in range(gas):
            # a fresh synthetic batch every micro-step (generated on the device: no H2D in the loop)
            batch = torch.randint(0, cfg.vocab_size, (mbs, seq), generator=gen, device=dev)
            if sp > 1:
                from shuffle_exchange_amd.sequence.data import shard_batch_for_sp
                b = shard_batch_for_sp(batch, sp_rank, sp)
                loss = engine(b["input_ids"], labels=b["labels"], position_ids=b["position_ids"], shift_labels=False)
            else:
                loss = engine(batch, labels=batch)
            engine.backward(loss)
            engine.step()
        return loss

    diag = None
    for i in range(args.warmup):
        if i == 0 and world > 1:  # collective fingerprint of the first step: every rank issued the same
            dist.reset_fingerprint()   # sequence of (op, group, size, dtype) or the run stops here
            dist.enable_fingerprint(True)
        loss = train_step()
        if i == 0 and world > 1:
            dist.enable_fingerprint(False)
            digest, count = dist.fingerprint_digest()
            try:  # a diagnostic: a mismatch is reported, it does not end the benchmark
                agree = bool(dist.verify_fingerprints())
            except RuntimeError as e:
                agree = False
                print(f"[bench] WARNING: {e}", file=sys.stderr, flush=True)
            it = dist.get_init_times()
            diag = {"fingerprint_first_step": {"sha1": digest[:16], "collectives": count, "ranks_agree": agree},
                    "init_process_group_ms": round(it["init_process_group_ms"] or 0.0, 1),
                    "communicators": len(it["groups"]),
                    "communicator_init_ms": round(sum(ms for _, ms in it["groups"]), 1),
                    "communicator_init_max_ms": round(max([ms for _, ms in it["groups"]] or [0.0]), 1)}
            if rank == 0:
                print(f"[bench] first step: {count} collectives, fingerprints {'agree' if agree else 'DIFFER'} on {world} ranks; "
                      f"init_process_group {diag['init_process_group_ms']} ms, {diag['communicators']} "
                      f"communicators in {diag['communicator_init_ms']} ms", file=sys.stderr, flush=True)
    sync()
    dist.barrier()
    sync()
    dist.reset_comms_stats()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = train_step()
    sync()
    dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    vol = dist.get_comm_volume()
    prof_dir = os.environ.get("SXE_BENCH_TORCH_PROFILE")
    if prof_dir and rank == 0 and on_gpu:  # one extra step AFTER the timed loop: kernel -> op -> Python stack
        _attribute_step(train_step, prof_dir)
    dist.barrier()
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    final_loss = loss.detach().float().reshape(1)
    if sp > 1:  # each SP rank holds its sequence shard's share of the loss: the sum is the sample loss
        dist.all_reduce(final_loss, group=groups.get_sequence_parallel_group())
    tokens = dp * mbs * gas * seq * args.steps
    tps = tokens / elapsed
    if c["family"] == "mixtral":
        d = cfg.hidden_size // cfg.num_attention_heads
        flops_tok = 6 * cfg.active_params_per_token() + 6 * cfg.num_hidden_layers * seq * cfg.num_attention_heads * d
    else:
        flops_tok = cfg.flops_per_token(seq)
    tflops = tps * flops_tok / world / 1e12
    full_model = layers is None
    valid = (full_model and model_name == c["model"] and stage == c["stage"] and on_gpu and seq == c["seq"]
             and mbs * gas == c["mbs"] * c["gas"])
    if rank == 0:
        model_tag = model_name + (f" ({layers} of {c['model']}'s layers)" if layers else "")
        par = [f"zero{stage}", f"dp{dp}"]
        if sp > 1:
            par.append(f"sp{sp}")
        if ep > 1:
            par.append(f"ep{ep}")
        if c.get("offload"):
            par.append("offload-optimizer-cpu")
        out = {
            "metric": c["metric"],
            "value": round(tps, 2),
            "unit": "tokens/s",
            "n_gpus": args.gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1000.0, 3),
            "higher_is_better": True,
            "scaling": "strong" if c.get("sp") else "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic",
            "config": {"name": args.config, "model": model_tag, "global_batch": dp * mbs * gas, "seq_len": seq,
                       "micro_batch_per_gpu": mbs, "grad_accum": gas, "parallelism": "-".join(par),
                       "params": n_params, "activation_checkpointing": (f"{policy}:{ac_layers}" if ac_layers is not None else policy) if ac else False,
                       "optimizer": "AdamW(fp32 master, " + ("C++ CPU Adam on host" if c.get("offload") else
                                                             "fused HIP") + ")",
                       "zero_knobs": c["knobs"], "zero_optimization": zero,
                       "zero_effective": effective_zero(engine.optimizer), "sequence_parallel_size": sp,
                       "expert_parallel_size": ep},
            "tflops_per_gpu": round(tflops, 1),
            "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2**30, 1) if on_gpu else None,
            "final_loss": round(float(final_loss.item()), 4),
            "comm_measured": {op: {"calls_per_step": round(n / args.steps, 2), "bytes_per_step": b // args.steps}
                              for op, (n, b) in sorted(vol.items())},
            "comm_model": comm_model(engine.optimizer, world, stage, c["knobs"], gas),
            "valid_for_metric": valid,
        }
        if diag is not None:
            out["diagnostics"] = diag
        print(json.dumps(out), flush=True)
    dist.barrier()
    if dist.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
