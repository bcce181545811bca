"""Task registry (parity: ``/root/reference/iit/tasks/task_loader.py:8-48``).

``get_dataset(task, dataset_config)`` -> ``(train IITDataset, test IITDataset)`` and
``get_alignment(task, config)`` -> ``(ll_model, hl_model, corr)`` for
``mnist_pvr`` / ``pvr_leaky``; ``ioi`` is registered too (the reference leaves it out).
"""
from __future__ import annotations

from typing import Tuple

from ..config import DEVICE
from ..data.iit_dataset import IITDataset
from .mnist_pvr.dataset import ImagePVRDataset
from .mnist_pvr.get_alignment import get_alignment as get_mnist_pvr_corr

DEFAULT_PVR_HOOK = "mod.layer3.mod.1.mod.conv2.hook_point"


def get_dataset(task: str, dataset_config: dict) -> Tuple[IITDataset, IITDataset]:
    if "pvr" in task:
        from .mnist_pvr import utils
        args = {"pad_size": 7, "train_size": 60000, "test_size": 10000, "device": DEVICE}
        args.update(dataset_config)
        if task not in ("mnist_pvr", "pvr_leaky"):
            raise ValueError(f"Unknown task {task}")
        dev = args["device"]
        train = ImagePVRDataset(utils.mnist_train, length=args["train_size"], pad_size=args["pad_size"],
                                unique_per_quad=False, device=dev)
        test = ImagePVRDataset(utils.mnist_test, length=args["test_size"], pad_size=args["pad_size"],
                               unique_per_quad=False, device=dev)
        return IITDataset(train, train, device=dev), IITDataset(test, test, device=dev)
    if task == "ioi":
        from .ioi import make_ioi_dataset_and_hl
        from ..data.iit_dataset import train_test_split
        dev = dataset_config.get("device", DEVICE)
        ds, _ = make_ioi_dataset_and_hl(dataset_config.get("num_samples", 12000), None, device=dev)
        tr, te = train_test_split(ds, test_size=0.2, random_state=42)
        return IITDataset(tr, tr, seed=0, device=dev), IITDataset(te, te, seed=0, device=dev)
    raise ValueError(f"Unknown task {task}")


def get_alignment(task: str, config: dict):
    if "pvr" in task:
        cfg = {"mode": "q", "hook_point": DEFAULT_PVR_HOOK, "model": "resnet18", "pad_size": 7}
        cfg.update(config)
        return get_mnist_pvr_corr(cfg, task)
    raise ValueError(f"Unknown task {task}")
