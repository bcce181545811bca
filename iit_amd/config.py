"""Global configuration (parity: ``/root/reference/iit/utils/config.py:1-4``).

``DEVICE`` is the *local* device of this process: ``cuda:<LOCAL_RANK>`` when a GPU
is visible (one process per MI355X, launched by ``torchrun``), else CPU.

Engine flags are read from the environment so scripts/benches can flip them
without code changes:

* ``IIT_BACKEND``   = ``hip`` | ``torch``  (default: hip when a GPU is present)
* ``IIT_DTYPE``     = ``bf16`` | ``fp32``  (compute dtype of the fast engine)
* ``IIT_PROFILE``   = 1 to emit roctx ranges / step timing
* ``IIT_DEBUG_SYNC``= 1 to serialise streams (race-debug mode)
"""
from __future__ import annotations

import os

import torch

WANDB_ENTITY = os.environ.get("IIT_WANDB_ENTITY", "cybershiptrooper")

if os.environ.get("IIT_DEBUG_SYNC", "0") == "1":
    # race-debug mode: the HIP runtime serialises kernel launches (read when HIP initialises, i.e. only if this
    # module is imported before the first GPU call -- ``import iit_amd`` does that); iit_amd.utils.tracing adds a
    # device drain at every phase boundary
    os.environ.setdefault("HIP_LAUNCH_BLOCKING", "1")
    os.environ.setdefault("AMD_SERIALIZE_KERNEL", "3")


def _local_device() -> torch.device:
    if torch.cuda.is_available():
        return torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count()))
    return torch.device("cpu")


DEVICE = _local_device()


def backend() -> str:
    b = os.environ.get("IIT_BACKEND")
    if b:
        return b
    return "hip" if torch.cuda.is_available() else "torch"


def compute_dtype() -> torch.dtype:
    return {"bf16": torch.bfloat16, "fp32": torch.float32}[os.environ.get("IIT_DTYPE", "bf16")]


def profiling_enabled() -> bool:
    return os.environ.get("IIT_PROFILE", "0") == "1"


def debug_sync() -> bool:
    return os.environ.get("IIT_DEBUG_SYNC", "0") == "1"
