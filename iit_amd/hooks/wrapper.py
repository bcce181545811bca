"""Give any ``nn.Module`` TL-style hook points (parity: ``/root/reference/iit/utils/wrapper.py:6-70``).

``HookedModuleWrapper(mod, name, recursive=True, hook_self=False)`` wraps every
child (ModuleLists element-wise) so that each child's output passes through a
``HookPoint``; hook names look like ``mod.layer3.mod.1.mod.conv2.hook_point``
exactly as in the reference (``/root/reference/iit/tasks/task_loader.py:41``).
"""
from __future__ import annotations

import torch
from torch import nn

from .hook_points import HookedRootModule, HookPoint

_TUPLE_RETURNING = ("intermediate_value_head", "value_head")


class HookedModuleWrapper(HookedRootModule):
    def __init__(self, mod: nn.Module, name: str = "model", recursive: bool = False, hook_self: bool = True,
                 top_level: bool = True, hook_pre: bool = False):
        super().__init__()
        self.mod = mod
        self.hook_self = hook_self
        self.hook_pre = None
        if hook_pre:
            self.hook_pre = HookPoint()
            self.hook_pre.name = name + "pre"
        if hook_self:
            self.hook_point = HookPoint()
            self.hook_point.name = name
        if recursive:
            self.wrap_hookpoints_recursively()
        self.setup()

    def wrap_hookpoints_recursively(self, verbose: bool = False) -> None:
        for key, child in list(self.mod._modules.items()):
            if child is None or isinstance(child, HookedModuleWrapper) or key in _TUPLE_RETURNING:
                continue
            if isinstance(child, nn.ModuleList):
                for i, sub in enumerate(child):
                    child[i] = HookedModuleWrapper(sub, name=f"{key}.{i}", recursive=True, top_level=False)
                continue
            setattr(self.mod, key, HookedModuleWrapper(child, name=key, recursive=True, top_level=False))

    def forward(self, *args, **kwargs):
        if self.hook_pre is not None:
            args = (self.hook_pre(args[0]),) + tuple(args[1:])
        out = self.mod(*args, **kwargs)
        if not self.hook_self:
            return out
        if not isinstance(out, torch.Tensor):
            raise TypeError(f"wrapped module returned {type(out)}, expected Tensor")
        return self.hook_point(out)


def get_hook_points(model: HookedRootModule):
    """Conv hook points of a wrapped CNN (parity: ``wrapper.py:69-70``)."""
    return [k for k in model.hook_dict.keys() if "conv" in k]
