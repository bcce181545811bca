"""Weight agreement after a few steps: single-GPU graphed schedule vs the data-parallel schedule on a one-rank RCCL
group (staged backward graphs, lazy zeroing), with and without the last-position final block.  Prints the largest
relative weight differences per comparison (diagnoses whether a mismatch is Adam-amplified noise or a lost update)."""
import os
import socket
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_dp_rccl_gpu import _train  # noqa: E402


def port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run(fast, dp, steps):
    from iit_amd.models import transformer
    transformer.HookedTransformer.last_position_final_block = fast
    if dp:
        os.environ["IIT_DP_FORCE_REDUCER"] = "1"
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port()}", rank=0, world_size=1)
    try:
        m, losses, _, _ = _train(steps)
    finally:
        if dp:
            dist.destroy_process_group()
            os.environ.pop("IIT_DP_FORCE_REDUCER")
    return {n: p.detach().float().clone() for n, p in m.named_parameters()}, losses


def cmp(tag, a, b):
    errs = sorted(((float((a[n] - b[n]).norm() / (a[n].norm() + 1e-12)), n) for n in a if not n.endswith("b_K")), reverse=True)
    print(f"{tag}: " + "  ".join(f"{n} {e:.2e}" for e, n in errs[:6]))
    n = errs[0][1]
    d = (a[n] - b[n]).abs().flatten()
    print(f"    {n}: {int((d > 5e-4).sum())} of {d.numel()} elements differ by > lr/2; largest diffs "
          f"{[round(float(x), 5) for x in d.topk(min(5, d.numel())).values]}")


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    r = {}
    for fast in (True, False):
        for dp in (False, True):
            r[(fast, dp)] = run(fast, dp, steps)
            print(fast, dp, r[(fast, dp)][1][-1], flush=True)
    cmp("single  fast vs full ", r[(True, False)][0], r[(False, False)][0])
    cmp("dp      fast vs full ", r[(True, True)][0], r[(False, True)][0])
    cmp("full    single vs dp ", r[(False, False)][0], r[(False, True)][0])
    cmp("fast    single vs dp ", r[(True, False)][0], r[(True, True)][0])


if __name__ == "__main__":
    main()
