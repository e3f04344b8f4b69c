"""Why does the packaged TunableOp table fail the ROCBLAS_VERSION validator? Print validators at
each stage and try read_file after different warm-ups."""
import sys
import torch
tun = torch.cuda.tunable
path = sys.argv[1]
tun.enable(True)
tun.tuning_enable(False)
print("validators before any GEMM:", tun.get_validators(), flush=True)
print("read_file #1:", tun.read_file(path), flush=True)
a = torch.ones(64, 64, device="cuda", dtype=torch.bfloat16)
torch.mm(a, a)
print("validators after bf16 mm:", tun.get_validators(), flush=True)
print("read_file #2:", tun.read_file(path), flush=True)
print("preferred blas:", torch.backends.cuda.preferred_blas_library(), flush=True)
prev = torch.backends.cuda.preferred_blas_library()
torch.backends.cuda.preferred_blas_library("cublas")
torch.mm(a, a)
torch.cuda.synchronize()
torch.backends.cuda.preferred_blas_library(prev)
print("validators after rocblas mm:", tun.get_validators(), flush=True)
print("read_file #3:", tun.read_file(path), flush=True)
print("results loaded:", len(tun.get_results()), flush=True)
