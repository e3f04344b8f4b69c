import time, torch
a = torch.randn(8192, 4096, device="cuda").to(torch.float8_e4m3fn)
b = torch.randn(4096, 4096, device="cuda").to(torch.float8_e4m3fn)
one = torch.ones((), device="cuda")
for name, kw in [("tensorwise", dict(scale_a=one, scale_b=one)),
                 ("rowwise", dict(scale_a=torch.ones(8192, 1, device="cuda"), scale_b=torch.ones(1, 4096, device="cuda")))]:
    try:
        out = torch._scaled_mm(a, b.t(), out_dtype=torch.bfloat16, **kw)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            out = torch._scaled_mm(a, b.t(), out_dtype=torch.bfloat16, **kw)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 20
        print(name, "ok", out.shape, f"{2*8192*4096*4096/dt/1e12:.0f} TF")
    except Exception as e:
        print(name, "FAILED", repr(e)[:300])
x = torch.randn(8192, 4096, device="cuda", dtype=torch.bfloat16); w = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
torch.cuda.synchronize(); t0 = time.perf_counter()
for _ in range(20): y = x @ w.t()
torch.cuda.synchronize(); print("bf16", f"{2*8192*4096*4096/((time.perf_counter()-t0)/20)/1e12:.0f} TF")
