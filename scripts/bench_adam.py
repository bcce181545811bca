"""Fused clip+Adam over a GPT-2-small-sized arena (124 M live parameters): bytes/s with and without
non-temporal moment/gradient streams (IIT_ADAM_NT) and 1 / 2 / 4 float4 groups per thread per pass
(IIT_ADAM_UNROLL), graph-timed."""
import os
import subprocess
import sys

CODE = r"""
import sys, torch
sys.path.insert(0, %r)
from iit_amd.engine.flat import FlatParams
from iit_amd.ops.optim import FusedAdam
n = 124_000_000
m = torch.nn.Linear(1, 1)
m.weight = torch.nn.Parameter(torch.randn(n // 4000, 4000, device="cuda") * 0.02)
m.bias = None
flat = FlatParams(m, with_bf16_shadow=True)
opt = FusedAdam(flat, lr=1e-4)
flat.grad.normal_()
opt.step(clip_norm=1.0)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    for _ in range(10):
        opt.step(clip_norm=1.0)
g.replay(); torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record(); g.replay(); e.record(); e.synchronize()
ms = s.elapsed_time(e) / 10
print(f"NT={os.environ.get('IIT_ADAM_NT', '1')} U={os.environ.get('IIT_ADAM_UNROLL', '1')}: {ms*1e3:8.1f} us per clip+Adam step, "
      f"{(n * 34) / (ms * 1e-3) / 1e12:5.2f} TB/s (34 B/param incl. the norm pass)")
""".replace("os.environ", "__import__('os').environ")

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for nt, u in (("1", "1"), ("1", "2"), ("1", "4"), ("0", "2"), ("1", "1"), ("1", "2"), ("1", "4")):
    out = subprocess.run([sys.executable, "-c", CODE % root], env=dict(os.environ, IIT_ADAM_NT=nt, IIT_ADAM_UNROLL=u),
                         capture_output=True, text=True, timeout=300)
    print(out.stdout.strip() or out.stderr[-500:])
