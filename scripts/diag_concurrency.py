"""Does MI355X run independent kernels of two streams concurrently -- eagerly, and inside a captured HIP graph?

Times the dX and dW GEMMs of one GPT-2-small MLP backward layer (T=4096 tokens) sequentially vs forked
onto a side stream.  Run once per HIP graph runtime setting (``--child`` re-runs this file with an env):
``DEBUG_CLR_GRAPH_PACKET_CAPTURE`` (packet capture replay) and ``DEBUG_HIP_FORCE_GRAPH_QUEUES``.
"""
import os
import subprocess
import sys

import torch

T, d, dm = 4096, 768, 3072


def child():
    dev = "cuda"
    g = torch.randn(T, dm, device=dev).bfloat16()
    x = torch.randn(T, d, device=dev).bfloat16()
    W = torch.randn(d, dm, device=dev).bfloat16()
    dW = torch.zeros(d, dm, device=dev)
    dx = torch.empty(T, d, device=dev, dtype=torch.bfloat16)
    tmp = torch.empty(d, dm, device=dev, dtype=torch.bfloat16)
    side = torch.cuda.Stream()

    def dx_op():
        torch.mm(g, W.t(), out=dx)

    def dw_op():
        torch.mm(x.t(), g, out=tmp)

    def seq():
        dx_op()
        dw_op()

    def par():
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            dw_op()
        dx_op()
        cur.wait_stream(side)

    def eager(fn, reps=200):
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        e.synchronize()
        return s.elapsed_time(e) / reps * 1e3

    def graphed(fn, reps=20):
        fn()
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for _ in range(reps):
                fn()
        gr.replay()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            gr.replay()
        e.record()
        e.synchronize()
        return s.elapsed_time(e) / (10 * reps) * 1e3

    tag = " ".join(f"{k}={os.environ[k]}" for k in ("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "DEBUG_HIP_FORCE_GRAPH_QUEUES")
                   if k in os.environ) or "default"
    print(f"[{tag}] dx only {eager(dx_op):6.1f} us  dw only {eager(dw_op):6.1f} us | eager seq {eager(seq):6.1f}"
          f"  eager 2-stream {eager(par):6.1f} | graph seq {graphed(seq):6.1f}  graph 2-stream {graphed(par):6.1f}",
          flush=True)


if __name__ == "__main__":
    if "--child" in sys.argv:
        child()
        sys.exit(0)
    envs = [{}, {"DEBUG_CLR_GRAPH_PACKET_CAPTURE": "0"}, {"DEBUG_HIP_FORCE_GRAPH_QUEUES": "2"},
            {"DEBUG_HIP_FORCE_GRAPH_QUEUES": "4"},
            {"DEBUG_CLR_GRAPH_PACKET_CAPTURE": "0", "DEBUG_HIP_FORCE_GRAPH_QUEUES": "4"}]
    rc = 0
    for extra in envs:
        r = subprocess.run([sys.executable, __file__, "--child"], env={**os.environ, **extra}, timeout=120)
        rc = rc or r.returncode
    sys.exit(rc)
