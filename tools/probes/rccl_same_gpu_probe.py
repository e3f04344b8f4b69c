"""Probe: can two RCCL ranks share one GPU (both on cuda:0)? NCCL refuses ('Duplicate GPU detected');
this records what RCCL on MI355X does. Run: torchrun --nproc-per-node 2 --master-addr 127.0.0.1 ..."""
import os

import torch
import torch.distributed as dist

torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
x = torch.full((1024,), float(dist.get_rank() + 1), device="cuda")
dist.all_reduce(x)
torch.cuda.synchronize()
print(f"rank {dist.get_rank()}: all_reduce -> {x[0].item()} (expected 3.0)", flush=True)
dist.destroy_process_group()
