"""Leakiness HL for PVR (parity: ``/root/reference/iit/tasks/mnist_pvr/pvr_check_leaky_hl.py:10-109``).

Twelve extra hooks ``hook_{i}_leaked_to_{j}`` (i != j quadrants) sit on quadrant
``i``'s digit; ``get_corr(mode="q", ...)`` aligns each with quadrant ``j``'s
spatial slice of an LL conv hook, asking whether information about digit ``i``
can be read from / ablated at digit ``j``'s location.
"""
from __future__ import annotations

import torch

from ...core.index import Ix
from ...core.nodes import HLNode, HookName, LLNode
from ...hooks.hook_points import HookedRootModule, HookPoint
from ..hl_model import HLModel
from .pvr_hl import MNIST_PVR_HL, _QUADS, hook_output_shape, quadrant_of
from .utils import MNIST_CLASS_MAP

_HOOK_STR = "hook_{}_leaked_to_{}"


class MNIST_PVR_Leaky_HL(HookedRootModule, HLModel):
    def __init__(self, class_map=MNIST_CLASS_MAP, device=None):
        super().__init__()
        self.hook_tl = HookPoint()
        self.hook_tr = HookPoint()
        self.hook_bl = HookPoint()
        self.hook_br = HookPoint()
        self.leaky_hooks = {}
        for i in _QUADS:
            for j in _QUADS:
                if i != j:
                    node = HLNode(_HOOK_STR.format(i, j), 10, None)
                    hp = HookPoint()
                    self.leaky_hooks[node] = hp
                    setattr(self, node.name, hp)
        self.register_buffer("class_map", torch.tensor([class_map[i] for i in range(len(class_map))],
                                                       dtype=torch.long, device=device or "cpu"))
        self.setup()

    def is_categorical(self) -> bool:
        return True

    def get_idx_to_intermediate(self, name: HookName):
        i = quadrant_of(name.split("_leaked_to_")[0])
        return lambda intermediate_vars: intermediate_vars[:, i]

    def forward(self, args):
        _, _, intermediate_data = args
        q = [intermediate_data[:, i] for i in range(4)]
        q = [self.hook_tl(q[0]), self.hook_tr(q[1]), self.hook_bl(q[2]), self.hook_br(q[3])]
        for node, hp in self.leaky_hooks.items():
            i = quadrant_of(node.name.split("_leaked_to_")[0])
            q[i] = hp(q[i])
        return MNIST_PVR_HL._select(self.class_map, *q)


_HL = None


def __getattr__(name):
    # the reference builds a module-level instance on DEVICE at import; build it lazily instead
    global _HL
    if name == "hl":
        if _HL is None:
            _HL = MNIST_PVR_Leaky_HL()
        return _HL
    raise AttributeError(name)


def get_corr(mode: str, hook_point: str, model: HookedRootModule, input_shape):
    if mode != "q":
        raise NotImplementedError(mode)
    return corr_for_shape(hook_point, hook_output_shape(model, hook_point, input_shape))


def corr_for_shape(hook_point: str, shape):
    """``get_corr(mode="q")`` for a hook whose output shape is already known."""
    assert shape[2] == shape[3], "Input shape is not square"
    h = shape[2] // 2
    idx = {"tl": Ix[None, None, :h, :h], "tr": Ix[None, None, :h, h:2 * h],
           "bl": Ix[None, None, h:2 * h, :h], "br": Ix[None, None, h:2 * h, h:2 * h]}
    corr = {}
    for i in _QUADS:
        for j in _QUADS:
            if i != j:
                corr[HLNode(_HOOK_STR.format(i, j), 10, None)] = {LLNode(name=hook_point, index=idx[j])}
    return corr
