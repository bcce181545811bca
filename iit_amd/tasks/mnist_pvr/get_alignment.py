"""LL model + HL model + correspondence for the PVR tasks (parity: ``/root/reference/iit/tasks/mnist_pvr/get_alignment.py``)."""
from __future__ import annotations

import torch

from ...config import DEVICE
from ...hooks.wrapper import HookedModuleWrapper
from ...models.resnet import resnet18
from .pvr_check_leaky_hl import MNIST_PVR_Leaky_HL
from .pvr_check_leaky_hl import get_corr as get_corr_leaky
from .pvr_hl import MNIST_PVR_HL, get_corr


def get_alignment(config, task):
    device = config.get("device", DEVICE)
    if config["model"] == "resnet18":
        net = resnet18()
        net.fc = torch.nn.Linear(512, 10)
        ll_model = HookedModuleWrapper(net, name="resnet18", recursive=True, hook_self=False).to(device)
    else:
        raise ValueError(f"Unknown model {config['model']}")
    if task == "mnist_pvr":
        hl_model = MNIST_PVR_HL().to(device)
        corr = get_corr(config["mode"], config["hook_point"], ll_model, config["input_shape"])
    elif task == "pvr_leaky":
        hl_model = MNIST_PVR_Leaky_HL().to(device)
        corr = get_corr_leaky(config["mode"], config["hook_point"], ll_model, config["input_shape"])
    else:
        raise ValueError(f"Unknown task {task}")
    return ll_model, hl_model, corr
