"""Is torch.addmm(C_fp32, A_bf16, B_bf16, out_dtype=fp32, out=C) (one hipBLASLt call, beta=1) available on ROCm?
Times it against mm(out fp32) + add_ for a Llama-3-8B weight-gradient shape (X^T dY, K = 384 tokens)."""
import torch

dev = "cuda"
for (M, N, K) in [(4096, 14336, 384), (4096, 4096, 384), (768, 3072, 4096)]:
    a = torch.randn(K, M, device=dev).bfloat16().t()
    b = torch.randn(K, N, device=dev).bfloat16()
    c = torch.zeros(M, N, device=dev)
    ok = True
    try:
        torch.addmm(c, a, b, out_dtype=torch.float32, out=c)
        ref = (a.float() @ b.float())
        err = ((c - ref).abs().max() / ref.abs().max()).item()
        print("addmm out_dtype aliasing OK, rel err", err)
    except Exception as e:
        ok = False
        print("addmm out_dtype failed:", type(e).__name__, str(e)[:200])
    try:
        r = torch.addmm(c, a, b, out_dtype=torch.float32)
        print("addmm out_dtype (no out) OK", r.dtype)
    except Exception as e:
        print("addmm out_dtype (no out) failed:", type(e).__name__, str(e)[:200])

    def t(fn, reps=20):
        fn(); torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record(); e.synchronize()
        return s.elapsed_time(e) / reps * 1e3
    t_mm_add = t(lambda: c.add_(torch.mm(a, b, out_dtype=torch.float32)))
    line = f"M={M} N={N} K={K}: mm+add {t_mm_add:.1f} us"
    if ok:
        line += f"  addmm beta=1 {t(lambda: torch.addmm(c, a, b, out_dtype=torch.float32, out=c)):.1f} us"
    print(line)
