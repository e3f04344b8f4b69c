"""Peak trainable parameters per GPU (the second half of BASELINE.json's headline metric).

Trains the Llama-3-70B architecture (hidden 8192, 64/8 heads, FFN 28672, vocab 128256) cut to L
decoder layers -- params = 0.856 B x L + 2.1 B -- with ZeRO-3 bf16 + AdamW (fp32 masters) and
activation checkpointing, seq 2048, micro-batch 1, for 2 full optimizer steps, for growing L in
fresh child processes, and reports the largest model that trains. Modes:
  hbm          everything in HBM (18 B/param + activations; 288 GB per MI355X)
  cpu_offload  ZeRO-Infinity host tier: fp32 master/m/v + bf16 staging in pinned host DRAM
               (14 B/param on the host, 6 B/param in HBM); sizes whose host need exceeds
               --host-gb are skipped, never attempted (the host must not run out of memory)
  --ratio r    Twin-Flow partial offload (cpu_offload only): the first r of every param group on the
               host (12 r B/param there), the rest stepped in HBM (6 + 12 (1 - r) B/param)
Usage: python tools/peak_params.py --mode hbm --layers 12,14,15
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def params_for(L):
    h, f, v, kv = 8192, 28672, 128256, 1024
    per_layer = h * (h + 2 * kv + h) + 3 * h * f + 2 * h
    return L * per_layer + 2 * v * h + h


def child(L, mode, seq, steps, ratio=1.0):
    sys.path.insert(0, ROOT)
    import torch
    import shuffle_exchange_amd as sxe
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    sxe.init_distributed(verbose=False)
    cfg = llama_config("llama3-70b", num_hidden_layers=L, activation_checkpointing=True,
                       max_position_embeddings=max(8192, seq))
    with sxe.zero.Init(dtype=torch.bfloat16):
        model = LlamaForCausalLM(cfg)
    zc = {"stage": 3, "stage3_param_persistence_threshold": 100_000, "reduce_bucket_size": 500_000_000}
    if mode == "cpu_offload":
        zc["offload_optimizer"] = {"device": "cpu", "pin_memory": True, "ratio": ratio}
    ds = {"train_micro_batch_size_per_gpu": 1, "gradient_accumulation_steps": 1, "bf16": {"enabled": True},
          "gradient_clipping": 1.0, "zero_optimization": zc,
          "optimizer": {"type": "AdamW", "params": {"lr": 1e-4, "weight_decay": 0.1}}, "steps_per_print": 10**9}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    n = sum(p.numel() for p in model.parameters())
    gen = torch.Generator(device="cuda").manual_seed(0)
    t0 = None
    for i in range(steps + 1):
        if i == 1:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        ids = torch.randint(0, cfg.vocab_size, (1, seq), generator=gen, device="cuda")
        loss = eng(ids, labels=ids)
        eng.backward(loss)
        eng.step()
        print(json.dumps({"progress": f"step {i}", "loss": float(loss)}), flush=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    import psutil
    print("RESULT " + json.dumps({"layers": L, "params": n, "params_B": round(n / 1e9, 2), "mode": mode,
                                  "offload_ratio": ratio if mode == "cpu_offload" else None,
                                  "peak_hbm_GB": round(torch.cuda.max_memory_allocated() / 1e9, 1),
                                  "host_rss_GB": round(psutil.Process().memory_info().rss / 1e9, 1),
                                  "s_per_step": round(dt, 2), "tokens_per_s": round(seq / dt, 1),
                                  "loss": float(loss)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="hbm", choices=["hbm", "cpu_offload"])
    ap.add_argument("--layers", default="12,14,15")
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--host-gb", type=float, default=200.0)
    ap.add_argument("--ratio", type=float, default=1.0)
    ap.add_argument("--timeout", type=int, default=420)
    ap.add_argument("--child", type=int, default=None)
    a = ap.parse_args()
    if a.child is not None:
        return child(a.child, a.mode, a.seq, a.steps, a.ratio)
    best = None
    for L in [int(x) for x in a.layers.split(",")]:
        n = params_for(L)
        host_need = (12 * a.ratio * n + 20e9) / 1e9  # masters + moments (+ runtime) on the host
        if a.mode == "cpu_offload" and host_need > a.host_gb:
            print(json.dumps({"layers": L, "params_B": round(n / 1e9, 2), "skipped": "host memory estimate "
                              f"{host_need:.0f} GB > --host-gb {a.host_gb}"}), flush=True)
            continue
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29700 + L), RANK="0", WORLD_SIZE="1",
                   LOCAL_RANK="0")
        proc = subprocess.Popen([sys.executable, "-u", __file__, "--mode", a.mode, "--seq", str(a.seq), "--steps",
                                 str(a.steps), "--ratio", str(a.ratio), "--child", str(L)], env=env, stdout=subprocess.PIPE,
                                stderr=subprocess.STDOUT, text=True)
        lines = []
        t_start = time.time()
        for ln in proc.stdout:  # stream the child's progress (keeps long runs visibly alive)
            lines.append(ln.rstrip())
            print(f"  [L={L}] {ln.rstrip()[:200]}", flush=True)
            if time.time() - t_start > a.timeout:
                proc.kill()
                break
        proc.wait()

        class _R:
            returncode = proc.returncode
            stdout = "\n".join(lines)
        p = _R()
        res = [ln[7:] for ln in p.stdout.splitlines() if ln.startswith("RESULT ")]
        if p.returncode == 0 and res:
            best = json.loads(res[-1])
            print(json.dumps(best), flush=True)
        else:
            tail = " | ".join(p.stdout.strip().splitlines()[-3:])[-400:]
            oom = "OutOfMemory" in p.stdout or "out of memory" in p.stdout
            print(json.dumps({"layers": L, "params_B": round(n / 1e9, 2), "failed": "OOM" if oom else
                              f"rc={p.returncode}", "tail": tail}), flush=True)
            if p.returncode < 0 or not oom:
                break  # a crash, not a capacity limit: stop here
            break
    print("PEAK " + json.dumps(best), flush=True)


if __name__ == "__main__":
    main()
