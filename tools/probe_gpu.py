"""Quick hardware probe: GEMM/SDPA throughput and memory on one MI355X."""
import time, torch, torch.nn.functional as F, json, os
d = torch.device("cuda:0")
p = torch.cuda.get_device_properties(0)
out = {"name": p.name, "mem_GB": p.total_memory/1e9, "cus": p.multi_processor_count, "arch": getattr(p, "gcnArchName", "")}
def bench(fn, n=20):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t=time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize(); return (time.perf_counter()-t)/n
for (m,n,k) in [(16384,4096,4096),(16384,14336,4096),(16384,4096,14336),(16384,6144,4096),(16384,128256,4096),(4096,14336,16384)]:
    a=torch.randn(m,k,device=d,dtype=torch.bfloat16); b=torch.randn(n,k,device=d,dtype=torch.bfloat16)
    t=bench(lambda: a@b.t()); out[f"gemm_{m}x{n}x{k}_TF"]=2*m*n*k/t/1e12
for (B,H,Hk,S,D) in [(8,32,8,2048,128),(2,32,8,8192,128)]:
    q=torch.randn(B,H,S,D,device=d,dtype=torch.bfloat16,requires_grad=True)
    k=torch.randn(B,H,S,D,device=d,dtype=torch.bfloat16,requires_grad=True)
    v=torch.randn(B,H,S,D,device=d,dtype=torch.bfloat16,requires_grad=True)
    t=bench(lambda: F.scaled_dot_product_attention(q,k,v,is_causal=True))
    fl=4*B*H*S*S*D/2
    out[f"sdpa_fwd_{B}x{H}x{S}_TF"]=fl/t/1e12
    o=F.scaled_dot_product_attention(q,k,v,is_causal=True); g=torch.randn_like(o)
    t=bench(lambda: torch.autograd.grad(F.scaled_dot_product_attention(q,k,v,is_causal=True),(q,k,v),g))
    out[f"sdpa_fwdbwd_{B}x{H}x{S}_TF"]=3.5*fl/t/1e12
x=torch.empty(2**30,device=d,dtype=torch.float32); y=torch.empty_like(x)
t=bench(lambda: y.copy_(x)); out["copy_GBs"]=2*4*2**30/t/1e9
print(json.dumps(out, indent=1))
os.makedirs("gpurun_out", exist_ok=True); json.dump(out, open("gpurun_out/probe.json","w"), indent=1)
