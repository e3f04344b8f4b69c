"""Tune every GEMM shape of the Llama-3-8B training step with PyTorch TunableOp (hipBLASLt + rocBLAS
solution search) on the MI355X and write the winners to a CSV that bench.py / the engine load.

Runs a 2-layer model (identical GEMM shapes to the 32-layer one) for one fwd+bwd micro-step with
tuning enabled. Prints a heartbeat so the box's silence watchdog sees progress.
"""
import os, sys, threading, time
out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/tunableop_llama3_8b.csv"
mbs = int(sys.argv[2]) if len(sys.argv) > 2 else 4
seq = int(sys.argv[3]) if len(sys.argv) > 3 else 2048
import torch
torch.cuda.tunable.enable(True)
torch.cuda.tunable.tuning_enable(True)
torch.cuda.tunable.set_filename(out)
torch.cuda.tunable.set_max_tuning_duration(40)
torch.cuda.tunable.set_max_tuning_iterations(30)
sys.path.insert(0, ".")
import shuffle_exchange_amd as sxe
from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
done = False
def beat():
    t0 = time.time()
    while not done:
        time.sleep(20); print(f"[tune] alive {time.time()-t0:.0f}s", flush=True)
threading.Thread(target=beat, daemon=True).start()
cfg = llama_config("llama3-8b", num_hidden_layers=2)
with sxe.zero.Init(dtype=torch.bfloat16):
    model = LlamaForCausalLM(cfg)
ds = {"train_micro_batch_size_per_gpu": mbs, "bf16": {"enabled": True}, "zero_optimization": {"stage": 3},
      "optimizer": {"type": "AdamW", "params": {"lr": 1e-4}}}
eng, _, _, _ = sxe.initialize(model=model, config=ds)
ids = torch.randint(0, cfg.vocab_size, (mbs, seq), device="cuda")
for i in range(2):
    loss = eng(ids, labels=ids); eng.backward(loss); eng.step()
    torch.cuda.synchronize(); print(f"[tune] step {i} done", flush=True)
torch.cuda.tunable.write_file()
done = True
print("[tune] wrote", out, flush=True)
