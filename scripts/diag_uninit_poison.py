"""Uninitialised-memory / lifetime probe for the paired forward and the staged backward.

The LN-xhat16 experiment of round 3 made ``tests/test_paired.py::test_paired_with_staged_backward_cuts`` see a W_U
gradient mismatch between the staged and the plain backward.  W_U's gradient is ``x^T dlogits`` with ``x`` the final
norm's output, so a mismatch there means the two FORWARDS differed -- and the only thing xhat16 changes is which
buffers stay alive (the LN context keeps the bf16 output instead of the fp32 input), i.e. what the caching allocator
hands to later ``torch.empty`` calls.  This script poisons the allocator (fills and frees blocks of many sizes with a
marker value) before each run and compares forward outputs and gradients across poison values, with and without
xhat16 and with and without the staged cuts: a difference names a kernel that reads memory it never wrote.

Prints one ``[poison]`` line per configuration.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from iit_amd.core.index import Ix  # noqa: E402

L, D, H, DH, DM, V, S, B = 4, 128, 4, 32, 512, 1000, 16, 32

SITES = [
    {"blocks.2.attn.hook_z": [Ix[:, :, 1]], "blocks.0.mlp.hook_post": [Ix[[None]]]},  # the staged test's sites
    {"blocks.0.attn.hook_z": [Ix[[None]]]},
    {"blocks.1.attn.hook_z": [Ix[:, :, 2]]},
    {"blocks.1.mlp.hook_post": [Ix[[None]]]},
    {"blocks.2.mlp.hook_post": [Ix[:, :, :64]]},
    {"blocks.3.attn.hook_z": [Ix[:, :, 1]]},
    {"blocks.3.mlp.hook_post": [Ix[:, -1, :128]]},
    {"blocks.2.mlp.hook_post": [Ix[2:5]]},
]


def _model():
    from iit_amd.models.transformer import HookedTransformer
    cfg = dict(n_layers=L, d_model=D, n_heads=H, d_head=DH, d_mlp=DM, n_ctx=S, d_vocab=V, act_fn="gelu_new",
               normalization_type="LNPre", device="cuda", dtype=torch.bfloat16, positional_embedding_type="standard")
    torch.manual_seed(0)
    m = HookedTransformer(cfg)
    m.set_op_backend("hip")
    return m


def poison(value: float) -> None:
    """Fill-and-free blocks of every size class the step allocates, so later ``torch.empty`` returns ``value``."""
    keep = []
    for n in (1 << 10, 1 << 12, 1 << 14, 1 << 16, 1 << 18, 1 << 20, 1 << 21, 1 << 22, 1 << 23, 1 << 24):
        for _ in range(24):
            keep.append(torch.full((n,), value, dtype=torch.float32, device="cuda"))
    torch.cuda.synchronize()
    del keep


def run(m, base, src, sites, w, logits, staged: bool):
    from iit_amd.engine.staged import StagedBackward
    m.zero_grad(set_to_none=True)
    st = StagedBackward(m, 4) if staged else None
    if st is not None:
        st.arm()
    try:
        out, _ = m.run_paired(base, src, sites, logits=logits)
        o = out[:, -1] if out.dim() == 3 else out
        (o.float() * w).sum().backward()
        if st is not None:
            for k in st.stages():
                st.run_stage(k)
    finally:
        if st is not None:
            st.release()
            st.disarm()
    torch.cuda.synchronize()
    grads = {k: p.grad.detach().float().clone() for k, p in m.named_parameters() if p.grad is not None}
    return o.detach().float().clone(), grads


def compare(a, b):
    oa, ga = a
    ob, gb = b
    worst = [("out", float((oa - ob).abs().max()), bool(torch.isfinite(oa).all() and torch.isfinite(ob).all()))]
    for k in ga:
        if k not in gb:
            worst.append((k, float("inf"), False))
            continue
        worst.append((k, float((ga[k] - gb[k]).abs().max()), bool(torch.isfinite(ga[k]).all())))
    bad = [x for x in worst if x[1] != 0.0 or not x[2]]
    return bad


def focused(cases):
    """The configurations that differed in the full sweep, every differing parameter listed top layer first (the
    first one in backward order is where the unwritten memory enters); ``IIT_*`` toggles come from the parent."""
    m = _model()
    g = torch.Generator(device="cuda").manual_seed(3)
    base = torch.randint(0, V, (B, S), device="cuda", generator=g)
    src = torch.randint(0, V, (B, S), device="cuda", generator=g)
    w = torch.randn(B, V, device="cuda", generator=g)
    tag = " ".join(f"{k}={v}" for k, v in sorted(os.environ.items()) if k.startswith("IIT_")) or "defaults"
    for si, logits in cases:
        # the first run of a configuration vs later ones too (first-call effects: GEMM autotuning, lazy state)
        order = [("0-first", 0.0), ("nan", float("nan")), ("1e4", 1e4), ("-1e4", -1e4), ("0-last", 0.0)]
        res = {}
        for name, pv in order:
            poison(pv)
            res[name] = run(m, base, src, SITES[si], w, logits, False)
        for name, _ in order[:-1]:
            bad = [x for x in compare(res[name], res["0-last"]) if x[1] > 1e-3 or not x[2]]
            print(f"[bisect] {tag} sites={si} logits={logits} poison={name} vs 0-last: " +
                  (", ".join(f"{k} {d:.3g}{'' if f else ' nonfinite'}" for k, d, f in reversed(bad)) or "equal"),
                  flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--keys":
        # which problem keys choose the s+hip candidate, then exclude it at one key at a time
        import re
        import subprocess
        r = subprocess.run([sys.executable, "-u", __file__, "--focused"], env=dict(os.environ, IIT_GEMM_TRACE="1"),
                           timeout=300, capture_output=True, text=True)
        print(r.stdout[-4000:], flush=True)
        keys = sorted({ln.split("] ", 1)[1].rsplit(" -> ", 1)[0] for ln in r.stdout.splitlines()
                       if ln.startswith("[gemm]") and ln.endswith("-> s+hip")})
        print(f"[keys] s+hip chosen at {len(keys)} problem keys: {keys}", flush=True)
        for k in keys:
            env = dict(os.environ, IIT_GEMM_EXCLUDE="s\\+hip@" + re.escape(k) + ";")
            rr = subprocess.run([sys.executable, "-u", __file__, "--focused"], env=env, timeout=300)
            if rr.returncode != 0:
                print(f"[keys] {k} exited {rr.returncode}", flush=True)
                if rr.returncode < 0 or rr.returncode >= 124:
                    break
        return
    if len(sys.argv) > 1 and sys.argv[1] == "--bisect":
        import subprocess
        toggles = [{}, {"IIT_GEMM_EXCLUDE": r"s\+hip"}, {"IIT_GEMM_EXCLUDE": r"(z\+)?glds\d+k\d+"},
                   {"IIT_GEMM_EXCLUDE": r"dual.*k\d+"}, {"IIT_GEMM_EXCLUDE": r"z\+.*"},
                   {"IIT_GEMM_EXCLUDE": r"s\+hip,(z\+)?glds\d+k\d+,dual.*k\d+"}]
        if len(sys.argv) > 2 and sys.argv[2] == "--wide":
            toggles += [{"IIT_DEFER_BIAS_SUMS": "0"}, {"IIT_GEMM_DUAL": "0"}, {"IIT_DETERMINISTIC": "1"}]
        for t in toggles:
            env = dict(os.environ, **t)
            r = subprocess.run([sys.executable, "-u", __file__, "--focused"], env=env, timeout=300)
            if r.returncode != 0:
                print(f"[bisect] {t} exited {r.returncode}", flush=True)
                if r.returncode < 0 or r.returncode >= 124:
                    break
        return
    if len(sys.argv) > 1 and sys.argv[1] == "--focused":
        focused([(1, "last"), (4, "last"), (1, "full")])
        return
    m = _model()
    g = torch.Generator(device="cuda").manual_seed(3)
    base = torch.randint(0, V, (B, S), device="cuda", generator=g)
    src = torch.randint(0, V, (B, S), device="cuda", generator=g)
    w = torch.randn(B, V, device="cuda", generator=g)
    n_bad = 0
    for xh in ("0", "1"):
        os.environ["IIT_LN_XHAT16"] = xh
        for si, sites in enumerate(SITES):
            for logits in ("last", "full"):
                res = {}
                for staged in (False, True):
                    for pv in (0.0, float("nan"), 1e4):
                        poison(pv)
                        res[(staged, pv)] = run(m, base, src, sites, w, logits, staged)
                ref = res[(False, 0.0)]
                for key, val in res.items():
                    bad = compare(val, ref)
                    tag = f"xhat16={xh} sites={si} logits={logits} staged={key[0]} poison={key[1]}"
                    if bad:
                        n_bad += 1
                        print(f"[poison] MISMATCH {tag}: " + ", ".join(f"{k} {d:.3g}{'' if f else ' nonfinite'}"
                                                                       for k, d, f in bad[:6]), flush=True)
                print(f"[poison] done xhat16={xh} sites={si} logits={logits}", flush=True)
    print(f"[poison] configurations with a difference: {n_bad}", flush=True)


if __name__ == "__main__":
    main()
