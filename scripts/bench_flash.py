"""Tiled MFMA attention (csrc/flash_attn.hip) vs torch SDPA and the materialised-softmax path on long sequences.

Prints forward and forward+backward time per call and attention TFLOP/s (causal counts half the S^2 work)."""
import math
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from iit_amd.ops import hip_ops  # noqa: E402

SHAPES = [  # B, S, Hq, Hkv, dh, causal
    (8, 1024, 12, 12, 64, True),    # GPT-2-small at n_ctx
    (4, 512, 12, 12, 64, False),    # BERT-base at 512
    (2, 2048, 32, 8, 128, True),    # Llama-3-8B heads at 2k
]


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    print(f"{'B':>3s} {'S':>5s} {'Hq':>3s} {'Hkv':>3s} {'dh':>4s} {'causal':>6s} | {'flash fwd':>10s} {'sdpa fwd':>10s} "
          f"{'flash f+b':>10s} {'sdpa f+b':>10s} | flash fwd TF/s  f+b TF/s")
    for B, S, Hq, Hkv, dh, causal in SHAPES:
        torch.manual_seed(0)
        q = torch.randn(B, S, Hq, dh, device="cuda").bfloat16().requires_grad_()
        k = torch.randn(B, S, Hkv, dh, device="cuda").bfloat16().requires_grad_()
        v = torch.randn(B, S, Hkv, dh, device="cuda").bfloat16().requires_grad_()
        g = torch.randn(B, S, Hq, dh, device="cuda").bfloat16()
        sc = math.sqrt(dh)

        def fl_f():
            with torch.no_grad():
                hip_ops.flash_attention(q, k, v, causal, sc)

        def fl_fb():
            hip_ops.flash_attention(q, k, v, causal, sc).backward(g)

        rep = Hq // Hkv
        qt = q.detach().transpose(1, 2).contiguous().requires_grad_()
        kt = k.detach().repeat_interleave(rep, 2).transpose(1, 2).contiguous().requires_grad_()
        vt = v.detach().repeat_interleave(rep, 2).transpose(1, 2).contiguous().requires_grad_()
        gt = g.transpose(1, 2).contiguous()

        def sd_f():
            with torch.no_grad():
                F.scaled_dot_product_attention(qt, kt, vt, is_causal=causal)

        def sd_fb():
            F.scaled_dot_product_attention(qt, kt, vt, is_causal=causal).backward(gt)

        tf, ts, tfb, tsb = timed(fl_f), timed(sd_f), timed(fl_fb), timed(sd_fb)
        flops = 4.0 * B * Hq * S * S * dh * (0.5 if causal else 1.0)
        print(f"{B:3d} {S:5d} {Hq:3d} {Hkv:3d} {dh:4d} {str(causal):>6s} | {tf:8.1f}us {ts:8.1f}us {tfb:8.1f}us "
              f"{tsb:8.1f}us | {flops / tf / 1e6:8.0f}  {3.5 * flops / tfb / 1e6:8.0f}")


if __name__ == "__main__":
    main()
