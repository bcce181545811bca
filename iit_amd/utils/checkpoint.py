"""Checkpoints: the reference's end-of-training layout + a separate full resume state.

Reference layout (``/root/reference/train_ioi.py:52-82``, ``eval_ioi.py:24-42``)::

    models/ioi/{PairClassName}/{int(100*behavior_weight)}_{int(100*iit_weight)}_{int(100*strict_weight)}/
        ll_model.pth         state_dict with TL parameter names/shapes (dense tensors)
        training_args.json   json of training_args (non-JSON values as str)
        ll_model_cfg.json    str(cfg.to_dict())  (a Python repr, as in the reference)
        metrics.log          epochs, early-stop flag, train/test metric values
        corr.json            {hl_hook: [ll_hook, ...]}

``metrics.log`` deliberately writes the metric *values* (the reference writes
``str(list_of_MetricStore)``, i.e. object reprs -- recorded as a deviation).

Resume state (not in the reference, which cannot resume) lives in separate files
so the layout above stays meaning-compatible:

    resume_state.pt      epoch, model/optimizer/scheduler state (rank 0)
    resume_rank{r}.pt    every RNG of rank r: torch CPU + GPU, numpy global, python
                         ``random``, and the pair's node-sampling ``np.random.Generator``
    resume_optim_rank{r}.pt  with a sharded optimizer (ZeRO-1, ``optimizer.sharded``):
                         rank r's own shard of the Adam moments (rank 0's file then
                         holds ``"optimizer": "sharded"`` instead of the state)

All files are written atomically (tmp + ``os.replace``) and read back with
``torch.load(weights_only=True)``.
"""
from __future__ import annotations

import json
import os
import random
from typing import Any, Dict, Optional

import numpy as np
import torch

from ..parallel import dist as pdist


# ----------------------------------------------------------------------------- helpers
def _atomic_torch_save(obj, path: str) -> None:
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def _atomic_text(path: str, text: str) -> None:
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        f.write(text)
    os.replace(tmp, path)


def dense_state_dict(module: torch.nn.Module) -> Dict[str, torch.Tensor]:
    """TL-keyed state dict of dense, independent tensors (arena-backed params are strided views)."""
    return {k: v.detach().clone().contiguous() for k, v in module.state_dict().items()}


def weights_dir_name(training_args: Dict[str, Any]) -> str:
    return (f"{int(100 * training_args.get('behavior_weight', 1.0))}_{int(100 * training_args.get('iit_weight', 1.0))}"
            f"_{int(100 * training_args.get('strict_weight', 0.0))}")


def model_dir(model_pair, root: str = "models/ioi") -> str:
    return os.path.join(root, type(model_pair).__name__, weights_dir_name(model_pair.training_args))


def _json_safe(d: Dict[str, Any]) -> Dict[str, Any]:
    out = {}
    for k, v in d.items():
        try:
            json.dumps(v)
            out[k] = v
        except TypeError:
            out[k] = str(v)
    return out


def _metric_lines(metrics) -> str:
    vals = []
    for m in metrics:
        v = m.get_value()
        if isinstance(v, np.ndarray):
            v = [round(float(x), 4) for x in v]
        elif v is not None:
            v = round(float(v), 4)
        vals.append(f"{m.get_name()}: {v}")
    return "[" + ", ".join(vals) + "]"


# ----------------------------------------------------------------------------- reference layout
def save_reference_layout(save_dir: str, model_pair, epochs: int, corr_dict: Optional[Dict] = None) -> str:
    """Write the reference's end-of-training files for ``model_pair`` under ``save_dir`` (rank 0 only)."""
    if not pdist.is_main():
        return save_dir
    os.makedirs(save_dir, exist_ok=True)
    ll = model_pair._ll_module() if hasattr(model_pair, "_ll_module") else model_pair.ll_model
    _atomic_torch_save(dense_state_dict(ll), os.path.join(save_dir, "ll_model.pth"))
    _atomic_text(os.path.join(save_dir, "training_args.json"), json.dumps(_json_safe(model_pair.training_args)))
    cfg = ll.cfg.to_dict() if hasattr(ll, "cfg") and hasattr(ll.cfg, "to_dict") else {}
    _atomic_text(os.path.join(save_dir, "ll_model_cfg.json"), str(cfg))
    test_metrics = getattr(model_pair, "test_metrics", None)
    train_metrics = getattr(model_pair, "train_metrics", None)
    lines = [f"Epochs: {epochs}"]
    if test_metrics is not None:
        try:
            stop = model_pair._check_early_stop_condition(test_metrics.metrics)
        except ValueError:
            stop = False
        lines.append(f"Early stop: {stop}")
    lines += ["", "", "--------------------------------", "", "Training metrics:",
              _metric_lines(train_metrics.metrics) if train_metrics is not None else "[]",
              "", "", "--------------------------------", "", "Test metrics:",
              _metric_lines(test_metrics.metrics) if test_metrics is not None else "[]"]
    _atomic_text(os.path.join(save_dir, "metrics.log"), "\n".join(lines))
    if corr_dict is None and hasattr(model_pair.corr, "to_name_dict"):
        corr_dict = model_pair.corr.to_name_dict()
    if corr_dict is not None:
        _atomic_text(os.path.join(save_dir, "corr.json"), json.dumps(corr_dict))
    return save_dir


def load_ll_model(save_dir: str, ll_model: torch.nn.Module) -> torch.nn.Module:
    path = os.path.join(save_dir, "ll_model.pth")
    if not os.path.exists(path):
        raise FileNotFoundError(f"Model not found at {save_dir}")
    dev = next(ll_model.parameters()).device
    ll_model.load_state_dict(torch.load(path, map_location=dev, weights_only=True))
    return ll_model


def load_corr(save_dir: str, suffixes=None, default=None):
    from ..core.correspondence import Correspondence
    path = os.path.join(save_dir, "corr.json")
    if os.path.exists(path):
        with open(path) as f:
            return Correspondence.make_corr_from_dict(json.load(f), suffixes=suffixes)
    print("WARNING: No corr.json found, using default corr_dict")
    return default


# ----------------------------------------------------------------------------- resume state
def _rng_state(model_pair) -> Dict[str, Any]:
    npst = np.random.get_state(legacy=False)
    npst = {**npst, "state": {"key": torch.from_numpy(npst["state"]["key"].astype(np.int64)),
                              "pos": int(npst["state"]["pos"])}}
    st: Dict[str, Any] = {
        "torch_cpu": torch.get_rng_state(),
        "numpy_global": npst,  # key array stored as a tensor: loadable with weights_only=True
        "python": random.getstate(),
    }
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        st["torch_cuda"] = torch.cuda.get_rng_state()
    rng = getattr(model_pair, "rng", None)
    if isinstance(rng, np.random.Generator):
        st["pair_rng"] = rng.bit_generator.state
    return st


def _set_rng_state(model_pair, st: Dict[str, Any]) -> None:
    torch.set_rng_state(st["torch_cpu"])
    npst = dict(st["numpy_global"])
    npst["state"] = {"key": npst["state"]["key"].numpy().astype(np.uint32), "pos": int(npst["state"]["pos"])}
    np.random.set_state(npst)
    random.setstate(_tuplify(st["python"]))
    if "torch_cuda" in st and torch.cuda.is_available():
        torch.cuda.set_rng_state(st["torch_cuda"])
    if "pair_rng" in st and isinstance(getattr(model_pair, "rng", None), np.random.Generator):
        model_pair.rng.bit_generator.state = st["pair_rng"]


def _tuplify(x):
    if isinstance(x, list):
        return tuple(_tuplify(v) for v in x)
    return x


def _is_sharded(optimizer) -> bool:
    return optimizer is not None and bool(getattr(optimizer, "sharded", False))


def _join_gathers(optimizer) -> None:
    wait = getattr(optimizer, "wait_gathers", None)  # ZeRO-1 deferred all-gathers (parallel/zero.py)
    if wait is not None:
        wait()


def save_resume_state(checkpoint_dir: str, model_pair, optimizer, lr_scheduler, epoch: int) -> None:
    """Every rank writes its RNG file (and, for a sharded optimizer, its own moment shard); rank 0 writes model +
    optimizer + scheduler + epoch."""
    os.makedirs(checkpoint_dir, exist_ok=True)
    _join_gathers(optimizer)
    r = pdist.rank()
    _atomic_torch_save(_rng_state(model_pair), os.path.join(checkpoint_dir, f"resume_rank{r}.pt"))
    sharded = _is_sharded(optimizer)
    if sharded:  # each rank owns different moments: one file per rank, never rank 0's shard for everyone
        _atomic_torch_save(optimizer.state_dict(), os.path.join(checkpoint_dir, f"resume_optim_rank{r}.pt"))
    if r == 0:
        ll = model_pair._ll_module() if hasattr(model_pair, "_ll_module") else model_pair.ll_model
        opt_state = None
        if optimizer is not None:
            opt_state = "sharded" if sharded else optimizer.state_dict()
        state = {"epoch": int(epoch), "world_size": pdist.world_size(), "model": dense_state_dict(ll),
                 "optimizer": opt_state,
                 "scheduler": lr_scheduler.state_dict() if lr_scheduler is not None else None}
        _atomic_torch_save(state, os.path.join(checkpoint_dir, "resume_state.pt"))


def has_resume_state(checkpoint_dir: str) -> bool:
    return os.path.exists(os.path.join(checkpoint_dir, "resume_state.pt"))


def load_resume_state(checkpoint_dir: str, model_pair, optimizer, lr_scheduler) -> int:
    """Restore a run saved by :func:`save_resume_state`; returns the epoch to continue from (0 if none)."""
    path = os.path.join(checkpoint_dir, "resume_state.pt")
    if not os.path.exists(path):
        return 0
    _join_gathers(optimizer)  # (an in-flight ZeRO-1 gather would land on the restored weights)
    ll = model_pair._ll_module() if hasattr(model_pair, "_ll_module") else model_pair.ll_model
    dev = next(ll.parameters()).device
    state = torch.load(path, map_location="cpu", weights_only=True)
    ll.load_state_dict({k: v.to(dev) for k, v in state["model"].items()})
    if optimizer is not None and state.get("optimizer") is not None:
        opt_sd = state["optimizer"]
        if opt_sd == "sharded" or _is_sharded(optimizer):
            if opt_sd != "sharded" or not _is_sharded(optimizer):
                raise ValueError("resume state: sharded and replicated optimizer states do not mix")
            opath = os.path.join(checkpoint_dir, f"resume_optim_rank{pdist.rank()}.pt")
            opt_sd = torch.load(opath, map_location="cpu", weights_only=True)
        if hasattr(optimizer, "flat"):
            opt_sd = {k: (v.to(dev) if torch.is_tensor(v) else v) for k, v in opt_sd.items()}
            optimizer.load_state_dict(opt_sd)
        else:
            optimizer.load_state_dict(opt_sd)
    if lr_scheduler is not None and state.get("scheduler") is not None:
        lr_scheduler.load_state_dict(state["scheduler"])
    rpath = os.path.join(checkpoint_dir, f"resume_rank{pdist.rank()}.pt")
    if os.path.exists(rpath):
        _set_rng_state(model_pair, torch.load(rpath, map_location="cpu", weights_only=True))
    if hasattr(ll, "mark_weights_changed"):
        ll.mark_weights_changed()
    flat = getattr(ll, "_flat_params", None)
    if flat is not None:
        flat.refresh_shadow()
    return int(state["epoch"])
