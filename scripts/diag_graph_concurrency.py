"""Does a captured HIP graph run independent branches concurrently on this ROCm?

Two independent GEMM chains (the backward's dX and dW shapes of GPT-2-small at 4096 tokens) are captured
(a) serially on one stream and (b) forked onto a side stream and joined, and both graphs are replayed and timed.
If (b) is faster than (a), graph branches overlap on the device and the engine can run weight-gradient GEMMs
beside the input-gradient chain.  Same test eagerly for reference.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from iit_amd.ops import hip_kernels as K
    from iit_amd.ops.gemm_dispatch import gemm

    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    T, d, dm = 4096, 768, 3072
    bf = torch.bfloat16
    g = torch.randn(T, d, device=dev, dtype=bf)        # dY of W_out
    W = torch.randn(dm, d, device=dev, dtype=bf)       # W_out [d_mlp][d]
    X = torch.randn(T, dm, device=dev, dtype=bf)       # post
    dx = torch.empty(T, dm, device=dev, dtype=bf)
    dW = torch.zeros(dm, d, device=dev, dtype=torch.float32)
    reps = int(os.environ.get("REPS", "8"))

    def dx_gemm():
        gemm(g, W, dx, M=T, N=dm, K=d, lda=d, ldb=d, ldc=dm, mode=K.MODE_NN, epi=K.EPI_BF16)

    def dw_gemm():
        gemm(X, g, dW, M=dm, N=d, K=T, lda=dm, ldb=d, ldc=d, mode=K.MODE_AKM | K.MODE_BKM, epi=K.EPI_F32_ACC)

    # settle autotuning outside capture
    for _ in range(3):
        dx_gemm()
        dw_gemm()
    torch.cuda.synchronize()

    side = torch.cuda.Stream()

    def serial():
        for _ in range(reps):
            dx_gemm()
            dw_gemm()

    def forked():
        cur = torch.cuda.current_stream()
        for _ in range(reps):
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                dw_gemm()
            dx_gemm()
            cur.wait_stream(side)

    def only_dx():
        for _ in range(reps):
            dx_gemm()

    def only_dw():
        for _ in range(reps):
            dw_gemm()

    def timed_graph(fn):
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            fn()
        gr.replay()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e9
        for _ in range(5):
            s.record()
            gr.replay()
            e.record()
            e.synchronize()
            best = min(best, s.elapsed_time(e) * 1e3 / reps)
        return best

    def timed_eager(fn):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e9
        for _ in range(5):
            s.record()
            fn()
            e.record()
            e.synchronize()
            best = min(best, s.elapsed_time(e) * 1e3 / reps)
        return best

    res = {}
    for name, fn in (("dx only", only_dx), ("dw only", only_dw), ("serial", serial), ("forked", forked)):
        res[name] = (timed_graph(fn), timed_eager(fn))
        print(f"{name:10s} graph {res[name][0]:8.1f} us/iter   eager {res[name][1]:8.1f} us/iter", flush=True)
    gain = res["serial"][0] / res["forked"][0]
    print(f"graph fork speedup over serial: {gain:.3f}x  (sum of parts {res['dx only'][0] + res['dw only'][0]:.1f} us)")
    print("HIP version", torch.version.hip)


if __name__ == "__main__":
    main()
