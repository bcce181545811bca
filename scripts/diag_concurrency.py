"""Does a captured HIP graph run independent kernels of forked streams concurrently on MI355X?
Times dX and dW GEMMs of one MLP layer (GPT-2-small backward shapes) sequentially vs on two streams."""
import torch

T, d, dm = 4096, 768, 3072
dev = "cuda"
g = torch.randn(T, dm, device=dev).bfloat16()
x = torch.randn(T, d, device=dev).bfloat16()
W = torch.randn(d, dm, device=dev).bfloat16()
dW = torch.zeros(d, dm, device=dev)
dx = torch.empty(T, d, device=dev, dtype=torch.bfloat16)
side = torch.cuda.Stream()


def seq():
    torch.mm(g, W.t(), out=dx)
    torch.addmm(dW, x.t(), g, out=dW, out_dtype=torch.float32) if False else dW.add_(torch.mm(x.t(), g).float())


def par():
    cur = torch.cuda.current_stream()
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        dW.add_(torch.mm(x.t(), g).float())
    torch.mm(g, W.t(), out=dx)
    cur.wait_stream(side)


def timed(fn, reps=20):
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
    for _ in range(5):
        gr.replay()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / (5 * reps) * 1e3


for _ in range(2):
    print(f"sequential {timed(seq):8.1f} us   two streams {timed(par):8.1f} us")
