"""HBM bandwidth reference points on this GPU (graph-timed): device-to-device copy and a 4-read / 3-write fp32
stream like the fused Adam's, to put the optimizer's bytes/s in context."""
import torch


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e-3


def main():
    n = 256 * 1024 * 1024  # 1 GiB of fp32 per tensor
    a, b = torch.randn(n, device="cuda"), torch.empty(n, device="cuda")
    t = timed(lambda: b.copy_(a))
    print(f"copy fp32 1 GiB -> 1 GiB: {2 * n * 4 / t / 1e12:5.2f} TB/s")
    m = n // 4
    p, g, mm, v = (torch.randn(m, device="cuda") for _ in range(4))

    def stream():  # read p, g, m, v; write p, m, v (torch fused elementwise: one pass per output)
        torch._foreach_add_([p, mm, v], [g, g, g])

    t = timed(stream)
    print(f"_foreach_add_ 3 outputs x (read 2, write 1): {3 * 3 * m * 4 / t / 1e12:5.2f} TB/s")


if __name__ == "__main__":
    main()
