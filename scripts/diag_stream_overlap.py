"""Does a memory-bound kernel on a second HIP stream run UNDER a compute-bound graph replay on the first?

The optimizer update (clip + Adam, ~0.58 ms per phase of the headline step, HBM-bound) could hide under the next
phase's forward GEMMs (MFMA-bound, HBM mostly idle) if the two actually share the chip.  Round 3 found that forked
branches INSIDE one captured graph serialise (profiles/graph_branch_concurrency_r3.txt).  This probe asks the
question one level up: graph A (a chain of forward GEMMs of the headline shapes) replayed on stream 1 while
graph B (Adam over ~10 M parameters, or a plain streaming copy) is replayed -- or launched eagerly -- on stream 2.

Prints per-case wall time (events on the main stream bracketing both streams) and the overlap ratio
(serial / concurrent).  A ratio near (tA + tB) / max(tA, tB) means real overlap.
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
    bf = torch.bfloat16
    M, d, n3, dm = 8192, 768, 2304, 3072
    x = torch.randn(M, d, device=dev, dtype=bf)
    # MODE_NN: A [M][K], B [N][K] (both k-contiguous)
    Wqkv = torch.randn(n3, d, device=dev, dtype=bf) * 0.02
    Win = torch.randn(dm, d, device=dev, dtype=bf) * 0.02
    Wout = torch.randn(d, dm, device=dev, dtype=bf) * 0.02
    qkv = torch.empty(M, n3, device=dev, dtype=bf)
    h = torch.empty(M, dm, device=dev, dtype=bf)
    y = torch.empty(M, d, device=dev, dtype=bf)
    layers = int(os.environ.get("LAYERS", "12"))

    def fwd_chain():
        for _ in range(layers):
            gemm(x, Wqkv, qkv, M=M, N=n3, K=d, lda=d, ldb=d, ldc=n3, mode=K.MODE_NN, epi=K.EPI_BF16)
            gemm(x, Win, h, M=M, N=dm, K=d, lda=d, ldb=d, ldc=dm, mode=K.MODE_NN, epi=K.EPI_BF16)
            gemm(h, Wout, y, M=M, N=d, K=dm, lda=dm, ldb=dm, ldc=d, mode=K.MODE_NN, epi=K.EPI_BF16)

    # memory-bound side job: Adam-shaped traffic (read p, g, m, v; write p, m, v) over P parameters, as torch ops
    # (foreach-free, a few large elementwise kernels) and as a plain streaming copy
    P = int(os.environ.get("PARAMS", str(124_000_000)))
    p = torch.randn(P, device=dev)
    g = torch.randn(P, device=dev) * 1e-3
    m = torch.zeros(P, device=dev)
    v = torch.zeros(P, device=dev)
    src = torch.randn(P, device=dev)
    dst = torch.empty(P, device=dev)

    def adam_like():
        m.mul_(0.9).add_(g, alpha=0.1)
        v.mul_(0.999).addcmul_(g, g, value=0.001)
        p.addcdiv_(m, v.sqrt().add_(1e-8), value=-1e-4)

    def copy_job():
        dst.copy_(src)

    for _ in range(3):
        fwd_chain()
        adam_like()
        copy_job()
    torch.cuda.synchronize()

    def cap(fn, stream=None):
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=stream):
            fn()
        gr.replay()
        torch.cuda.synchronize()
        return gr

    side = torch.cuda.Stream()
    gA = cap(fwd_chain)
    gB = cap(adam_like)
    gC = cap(copy_job)
    main_s = torch.cuda.current_stream()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fork = torch.cuda.Event()
    join = torch.cuda.Event()

    def timed(fn, reps=7):
        fn()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(reps):
            ev0.record(main_s)
            fn()
            ev1.record(main_s)
            ev1.synchronize()
            best = min(best, ev0.elapsed_time(ev1) * 1e3)
        return best

    def conc(side_fn):
        def run():
            fork.record(main_s)
            side.wait_event(fork)
            with torch.cuda.stream(side):
                side_fn()
            gA.replay()
            join.record(side)
            main_s.wait_event(join)
        return run

    res = {}
    res["fwd gemms (graph)"] = tA = timed(gA.replay)
    res["adam-like (graph)"] = tB = timed(gB.replay)
    res["copy (graph)"] = tC = timed(gC.replay)
    res["serial fwd+adam"] = timed(lambda: (gA.replay(), gB.replay()))
    res["conc fwd || adam graph on side stream"] = tAB = timed(conc(gB.replay))
    res["conc fwd || adam eager on side stream"] = tABe = timed(conc(adam_like))
    res["conc fwd || copy graph on side stream"] = tAC = timed(conc(gC.replay))
    for k, t in res.items():
        print(f"{k:42s} {t:9.1f} us", flush=True)
    print(f"adam: serial/concurrent = {(tA + tB) / tAB:.3f} (ideal {(tA + tB) / max(tA, tB):.3f}); "
          f"eager side {(tA + tB) / tABe:.3f}")
    print(f"copy: serial/concurrent = {(tA + tC) / tAC:.3f} (ideal {(tA + tC) / max(tA, tC):.3f})")
    print("HIP", torch.version.hip, "GPU_MAX_HW_QUEUES", os.environ.get("GPU_MAX_HW_QUEUES"))


if __name__ == "__main__":
    main()
