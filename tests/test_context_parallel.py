"""Context-parallel attention (iit_amd/parallel/context.py): a sequence sharded over a gloo group of 2 ranks gives the
same output and the same Q/K/V gradients as single-process attention over the whole sequence."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from iit_amd.parallel.context import context_parallel_attention, shard_sequence


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _reference(q, k, v, causal):
    H, Hkv = q.shape[2], k.shape[2]
    k = k.repeat_interleave(H // Hkv, dim=2)
    v = v.repeat_interleave(H // Hkv, dim=2)
    out = torch.nn.functional.scaled_dot_product_attention(
        q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), is_causal=causal)
    return out.transpose(1, 2)


def _inputs(Hkv):
    g = torch.Generator().manual_seed(0)
    B, S, H, D = 2, 12, 4, 8
    q = torch.randn(B, S, H, D, generator=g, dtype=torch.float64)
    k = torch.randn(B, S, Hkv, D, generator=g, dtype=torch.float64)
    v = torch.randn(B, S, Hkv, D, generator=g, dtype=torch.float64)
    w = torch.randn(B, S, H, D, generator=g, dtype=torch.float64)
    return q, k, v, w


def _worker(rank, world, port, causal, Hkv, out_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q, k, v, w = _inputs(Hkv)
        ql, kl, vl = (shard_sequence(t, 1).clone().requires_grad_(True) for t in (q, k, v))
        z = context_parallel_attention(ql, kl, vl, causal=causal)
        (z * shard_sequence(w, 1)).sum().backward()
        qr, kr, vr = (t.clone().requires_grad_(True) for t in (q, k, v))
        zr = _reference(qr, kr, vr, causal)
        (zr * w).sum().backward()
        checks = [(z, shard_sequence(zr, 1)), (ql.grad, shard_sequence(qr.grad, 1)),
                  (kl.grad, shard_sequence(kr.grad, 1)), (vl.grad, shard_sequence(vr.grad, 1))]
        ok = all(torch.allclose(a, b, atol=1e-9, rtol=1e-7) for a, b in checks)
        with open(os.path.join(out_dir, f"r{rank}"), "w") as f:
            f.write("ok" if ok else "mismatch " + " ".join(f"{(a - b).abs().max().item():.3g}" for a, b in checks))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("causal,Hkv", [(True, 4), (False, 4), (True, 2)])
def test_context_parallel_attention_matches_full_sequence(tmp_path, causal, Hkv):
    mp.spawn(_worker, args=(2, _free_port(), causal, Hkv, str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        assert (tmp_path / f"r{r}").read_text() == "ok", (tmp_path / f"r{r}").read_text()


def test_single_rank_is_plain_attention():
    q, k, v, _ = _inputs(4)
    assert torch.allclose(context_parallel_attention(q, k, v, causal=True), _reference(q, k, v, True), atol=1e-10)
