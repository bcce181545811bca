"""PVR high-level model and its correspondences (parity: ``/root/reference/iit/tasks/mnist_pvr/pvr_hl.py:10-134``).

``MNIST_PVR_HL`` exposes one hook per quadrant digit (``hook_tl/tr/bl/br``) and
returns the pointed-to digit: ``stack([tr, bl, br])[class_map[tl] - 1]``.
``get_corr(mode, hook_point, model, input_shape)`` aligns each quadrant with a
slice of one LL conv hook: a quarter of the channels (``mode="c"``) or the
matching spatial quadrant (``mode="q"``); the hook's output shape comes from a
dummy forward.
"""
from __future__ import annotations

import torch

from ...config import DEVICE
from ...core.index import Ix
from ...core.nodes import HLNode, HookName, LLNode
from ...hooks.hook_points import HookedRootModule, HookPoint
from ..hl_model import HLModel
from .utils import MNIST_CLASS_MAP

_QUADS = ("tl", "tr", "bl", "br")


def quadrant_of(name: str) -> int:
    for i, q in enumerate(_QUADS):
        if f"hook_{q}" in name:
            return i
    raise ValueError(f"Hook name {name} not recognised")


class MNIST_PVR_HL(HookedRootModule, HLModel):
    def __init__(self, class_map=MNIST_CLASS_MAP, device=None):
        super().__init__()
        self.hook_tl = HookPoint()
        self.hook_tr = HookPoint()
        self.hook_bl = HookPoint()
        self.hook_br = HookPoint()
        self.register_buffer("class_map", torch.tensor([class_map[i] for i in range(len(class_map))],
                                                       dtype=torch.long, device=device or "cpu"))
        self.setup()

    def is_categorical(self) -> bool:
        return True

    def get_idx_to_intermediate(self, name: HookName):
        if name not in ("hook_tl", "hook_tr", "hook_bl", "hook_br"):
            raise NotImplementedError(name)
        i = quadrant_of(name)
        return lambda intermediate_vars: intermediate_vars[:, i]

    def _quads(self, intermediate_data):
        tl, tr, bl, br = (intermediate_data[:, i] for i in range(4))
        return self.hook_tl(tl), self.hook_tr(tr), self.hook_bl(bl), self.hook_br(br)

    @staticmethod
    def _select(class_map, tl, tr, bl, br):
        pointer = class_map.to(tl.device)[tl] - 1
        return torch.stack([tr, bl, br], dim=0).gather(0, pointer.unsqueeze(0)).squeeze(0)

    def forward(self, args):
        _, _, intermediate_data = args
        tl, tr, bl, br = self._quads(intermediate_data)
        return self._select(self.class_map, tl, tr, bl, br)


hl_nodes = {f"hook_{q}": HLNode(f"hook_{q}", 10, None) for q in _QUADS}


def hook_output_shape(model: HookedRootModule, hook_point: str, input_shape) -> torch.Size:
    dev = next(model.parameters()).device if any(True for _ in model.parameters()) else torch.device(DEVICE)
    with torch.no_grad():
        _, cache = model.run_with_cache(torch.zeros(tuple(input_shape), device=dev))
    return cache[hook_point].shape


def get_corr(mode: str, hook_point: str, model: HookedRootModule, input_shape):
    shape = hook_output_shape(model, hook_point, input_shape)
    channels, side = shape[1], shape[2]
    assert shape[2] == shape[3], f"Input shape is not square, got {shape}"
    if mode == "c":
        cs = channels // 4
        return {hl_nodes[f"hook_{q}"]: {LLNode(hook_point, Ix[None, cs * i: cs * (i + 1), None, None])}
                for i, q in enumerate(_QUADS)}
    if mode == "q":
        h = side // 2
        spans = {"tl": (slice(0, h), slice(0, h)), "tr": (slice(0, h), slice(h, 2 * h)),
                 "bl": (slice(h, 2 * h), slice(0, h)), "br": (slice(h, 2 * h), slice(h, 2 * h))}
        return {hl_nodes[f"hook_{q}"]: {LLNode(hook_point, Ix[None, None, spans[q][0], spans[q][1]])}
                for q in _QUADS}
    raise ValueError(f"unknown mode {mode}")
