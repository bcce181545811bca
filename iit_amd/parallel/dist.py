"""Process-group plumbing: one process per MI355X, RCCL over xGMI.

``torch.distributed`` backend ``"nccl"`` *is* RCCL on ROCm.  ``init_distributed``
reads the torchrun env (``RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*``), binds the
process to ``cuda:LOCAL_RANK`` and falls back to ``gloo`` on CPU (the CPU test
path).  Rendezvous defaults to 127.0.0.1.
"""
from __future__ import annotations

import datetime
import os
from typing import Optional

import torch
import torch.distributed as dist


def is_initialized() -> bool:
    return dist.is_available() and dist.is_initialized()


def rank() -> int:
    return dist.get_rank() if is_initialized() else 0


def world_size() -> int:
    return dist.get_world_size() if is_initialized() else 1


def is_main() -> bool:
    return rank() == 0


def force_reducer() -> bool:
    """``IIT_DP_FORCE_REDUCER=1`` under a one-rank process group: run the full data-parallel machinery (RCCL
    all-reduces between staged graph replays) on a single GPU -- the rehearsal of the multi-GPU path that a
    one-GPU box can run (``scripts/dp_rccl_rehearsal.sh``)."""
    return os.environ.get("IIT_DP_FORCE_REDUCER") == "1" and is_initialized()


def local_device_index() -> int:
    """GPU of this rank: ``LOCAL_RANK``, or 0 for every rank under ``IIT_REHEARSE_ONE_GPU=1`` -- the rehearsal of the
    multi-rank data-parallel schedule on a one-GPU box (ranks share the card; pair it with
    ``IIT_DIST_BACKEND=gloo``, since RCCL refuses two ranks on one device)."""
    if os.environ.get("IIT_REHEARSE_ONE_GPU") == "1":
        return 0
    return int(os.environ.get("LOCAL_RANK", "0"))


def init_distributed(backend: Optional[str] = None, timeout_s: int = 600) -> bool:
    """Initialise the default process group from torchrun env vars. Returns True if distributed."""
    if is_initialized():
        return True
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1 and not (os.environ.get("IIT_DP_FORCE_REDUCER") == "1" and "RANK" in os.environ):
        return False
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    if backend is None:
        backend = os.environ.get("IIT_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if torch.cuda.is_available():
        torch.cuda.set_device(local_device_index())
    if backend == "nccl":
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    timeout = datetime.timedelta(seconds=timeout_s)
    attempt = int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0") or 0)
    if attempt > 0 and os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True":
        # a torchrun restart (--max-restarts): the agent's TCPStore outlives the failed attempt, and
        # its keys (the dead ranks' gloo / RCCL bootstrap addresses) would be read back by the new ranks -- the
        # restarted job rendezvouses under a per-attempt key prefix instead
        store = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), ws, is_master=False,
                              timeout=timeout)
        dist.init_process_group(backend=backend, store=dist.PrefixStore(f"iit/attempt_{attempt}", store),
                                rank=int(os.environ["RANK"]), world_size=ws, timeout=timeout)
        return True
    dist.init_process_group(backend=backend, timeout=timeout)
    return True


def barrier():
    if is_initialized():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def broadcast_module(module: torch.nn.Module, src: int = 0) -> None:
    """Make every rank start from rank ``src``'s parameters and buffers."""
    if not is_initialized() or world_size() == 1:
        return
    flat = getattr(module, "_flat_params", None)
    with torch.no_grad():
        tensors = list(module.buffers())
        if flat is not None:  # one collective over the whole arena (params are strided views of it)
            dist.broadcast(flat.data, src)
            module._iit_weights_version = getattr(module, "_iit_weights_version", 0) + 1
            tensors += [p for p in module.parameters() if not flat.owns(p)]
        else:
            tensors += list(module.parameters())
        for t in tensors:
            if t.is_contiguous():
                dist.broadcast(t.data, src)
            else:
                tmp = t.data.contiguous()
                dist.broadcast(tmp, src)
                t.data.copy_(tmp)


def all_reduce_mean_(t: torch.Tensor) -> torch.Tensor:
    if is_initialized() and world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        t.div_(world_size())
    return t


def destroy():
    if is_initialized():
        dist.destroy_process_group()
