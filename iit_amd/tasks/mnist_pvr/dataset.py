"""MNIST pointer-value-retrieval images (parity: ``/root/reference/iit/tasks/mnist_pvr/dataset.py:11-195``).

Item ``i`` tiles four digits (each padded by ``pad_size`` black pixels) into a 2x2
RGB image; the label is the digit in the quadrant that ``class_map[top-left digit]``
points to (1 = top-right, 2 = bottom-left, 3 = bottom-right).  The four source
digits of item ``i`` are drawn from ``default_rng(seed*length + i)`` exactly as
in the reference, so items are identical for the same base dataset.

MI355X-first data path: besides the per-item ``__getitem__`` (reference
semantics), :meth:`gather` assembles a whole batch on the device from the
HBM-resident uint8 digit array and a precomputed ``[length, 4]`` quadrant
table -- one gather + pad + concat, no PIL, no per-sample Python -- so
:class:`iit_amd.data.iit_dataset.DeviceIITLoader` can stream PVR pairs.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch
from torch.utils.data import Dataset

from ...config import DEVICE
from ...core.index import Index, Ix
from ...core.nodes import HLNode
from .utils import MNIST_CLASS_MAP


def _digit_tensor(base_dataset) -> torch.Tensor:
    data = getattr(base_dataset, "data", None)
    if isinstance(data, torch.Tensor) and data.dim() == 3:
        return data
    imgs = [np.array(base_dataset[i][0].convert("L"), dtype=np.uint8) for i in range(len(base_dataset))]
    return torch.from_numpy(np.stack(imgs))


def _targets(base_dataset) -> torch.Tensor:
    t = getattr(base_dataset, "targets", None)
    if t is not None:
        return torch.as_tensor(t, dtype=torch.long)
    return torch.tensor([int(base_dataset[i][1]) for i in range(len(base_dataset))], dtype=torch.long)


class ImagePVRDataset(Dataset):
    def __init__(self, base_dataset, class_map: Dict[int, int] = MNIST_CLASS_MAP, seed: int = 0, use_cache: bool = True,
                 length: int = 200000, iid: bool = True, pad_size: int = 0, unique_per_quad: bool = False,
                 device=None):
        assert all(v in {1, 2, 3} for v in class_map.values())
        self.base_dataset = base_dataset
        self.class_map = class_map
        self.seed = seed
        self.rng = np.random.default_rng(seed)
        self.use_cache = use_cache
        self.cache = {}
        self.length = length
        self.iid = iid
        self.pad_size = pad_size
        self.unique_per_quad = unique_per_quad
        self.device = torch.device(device) if device is not None else torch.device(DEVICE)
        if not self.iid:
            print("WARNING: using non-iid mode")
            assert len(self.base_dataset) >= 4 * self.length, "Dataset is too small for non-iid mode"
        self._quad: Optional[np.ndarray] = None
        self._dev_cache = {}
        self._class_map_t = torch.tensor([class_map[i] for i in range(len(class_map))], dtype=torch.long)
        self.input_shape = None
        side = 2 * (self._digit_side() + 2 * pad_size)
        self.set_input_shape(torch.Size([1, 3, side, side]))

    # ------------------------------------------------------------------ shapes
    def _digit_side(self) -> int:
        data = getattr(self.base_dataset, "data", None)
        if isinstance(data, torch.Tensor):
            return int(data.shape[-1])
        return self.base_dataset[0][0].size[0]

    def set_input_shape(self, shape):
        self.input_shape = shape

    def get_input_shape(self):
        return self.input_shape

    # ------------------------------------------------------------------ item sampling
    def quad_indices(self, index: int) -> np.ndarray:
        """The four base-dataset indices of item ``index`` (reference RNG call sequence)."""
        n = len(self.base_dataset)
        if not self.iid:
            return np.arange(index * 4, index * 4 + 4)
        self.rng = np.random.default_rng(self.seed * self.length + index)
        q = np.array([self.rng.integers(0, n) for _ in range(4)], dtype=np.int64)
        if self.unique_per_quad:
            tg = _targets(self.base_dataset)
            while len(set(int(tg[j]) for j in q)) < 4:
                q = np.array([self.rng.integers(0, n) for _ in range(4)], dtype=np.int64)
        return q

    def quad_table(self) -> np.ndarray:
        if self._quad is None:
            self._quad = np.stack([self.quad_indices(i) for i in range(self.length)]).astype(np.int64)
        return self._quad

    def make_label_from_intermediate(self, intermediate_vars: torch.Tensor) -> torch.Tensor:
        pointer = self.class_map[int(intermediate_vars[0])]
        return torch.tensor(int(intermediate_vars[pointer]))

    # ------------------------------------------------------------------ images
    def _assemble(self, digits: torch.Tensor) -> torch.Tensor:
        """[B, 4, s, s] uint8 -> [B, 3, H, W] float in [0, 1] (pad, 2x2 tile, gray->RGB)."""
        x = digits.float() / 255.0
        p = self.pad_size
        if p > 0:
            x = torch.nn.functional.pad(x, (p, p, p, p))
        top = torch.cat([x[:, 0], x[:, 1]], dim=-1)
        bottom = torch.cat([x[:, 2], x[:, 3]], dim=-1)
        img = torch.cat([top, bottom], dim=-2)
        return img.unsqueeze(1).expand(-1, 3, -1, -1).contiguous()

    def __getitem__(self, index):
        if self.use_cache and index in self.cache:
            return self.cache[index]
        q = torch.as_tensor(self.quad_indices(index))
        data = _digit_tensor(self.base_dataset)
        tg = _targets(self.base_dataset)
        img = self._assemble(data[q].unsqueeze(0))[0]
        iv = tg[q].clone()
        label = self.make_label_from_intermediate(iv)
        ret = (img, label, iv)
        if self.use_cache:
            self.cache[index] = ret
        return ret

    def __len__(self) -> int:
        return self.length

    def _device_state(self, dev):
        st = self._dev_cache.get(dev)
        if st is None:
            st = self._dev_cache[dev] = (_digit_tensor(self.base_dataset).to(dev), _targets(self.base_dataset).to(dev),
                                         torch.as_tensor(self.quad_table()).to(dev), self._class_map_t.to(dev))
        return st

    def gather(self, idx: torch.Tensor):
        """Batch ``(x [B,3,H,W], y [B], iv [B,4])`` for item indices ``idx``, built on ``idx.device``."""
        data, tg, quad, cmap = self._device_state(idx.device)
        q = quad.index_select(0, idx)  # [B, 4]
        iv = tg[q]  # [B, 4]
        x = self._assemble(data[q])
        y = iv.gather(1, cmap[iv[:, 0]].unsqueeze(1)).squeeze(1)
        return x, y, iv

    # ------------------------------------------------------------------ input-space patching (leakiness evals)
    def get_idx_and_intermediate(self, hl_node: HLNode):
        input_shape = self.get_input_shape()
        width, height = input_shape[2], input_shape[3]
        if "hook_tl" in hl_node.name:
            return Ix[None, : width // 2, : height // 2], 0
        if "hook_tr" in hl_node.name:
            return Ix[None, : width // 2, height // 2: height], 1
        if "hook_bl" in hl_node.name:
            return Ix[None, width // 2: width, : height // 2], 2
        if "hook_br" in hl_node.name:
            return Ix[None, width // 2: width, height // 2: height], 3
        raise ValueError(f"Hook name {hl_node.name} not recognised")

    def _quad_image(self, j: int, device) -> torch.Tensor:
        data = _digit_tensor(self.base_dataset)
        x = data[j].float().to(device) / 255.0
        if self.pad_size > 0:
            x = torch.nn.functional.pad(x, (self.pad_size,) * 4)
        return x.unsqueeze(0).expand(3, -1, -1)

    def patch_at_hl_idx(self, input: torch.Tensor, intermediate_var: torch.Tensor, idx: Index,
                        idx_to_intermediate: int):
        """Replace one quadrant with a random digit of a *different* class; returns (input, ivs, label)."""
        tg = _targets(self.base_dataset)
        new_input = input.clone().detach()
        while True:
            j = int(self.rng.integers(0, len(self.base_dataset)))
            quad_label = int(tg[j])
            if quad_label != int(intermediate_var[idx_to_intermediate]):
                new_input[idx.as_index] = self._quad_image(j, input.device)
                new_iv = intermediate_var.clone().detach()
                new_iv[idx_to_intermediate] = quad_label
                return new_input, new_iv, self.make_label_from_intermediate(new_iv)

    def patch_batch_tensor(self, x: torch.Tensor, intermediate_vars: torch.Tensor, hl_node: HLNode):
        """:meth:`patch_batch_at_hl` on whole tensors (``x`` [B,3,H,W], ``intermediate_vars`` [B,4]): the same draws
        from ``self.rng`` in the same order (so the same patches), then one gather + one slice write on the device
        instead of a per-sample Python loop of image copies.  Returns ``(x', labels' [B], ivs' [B,4])``."""
        idx, k = self.get_idx_and_intermediate(hl_node)
        js = self.draw_patch_digits(intermediate_vars[:, k].cpu().numpy())
        return self.apply_patch_digits(x, intermediate_vars, hl_node, js)

    def draw_patch_digits(self, cur: np.ndarray) -> np.ndarray:
        """The base-dataset indices :meth:`patch_at_hl_idx` draws for a batch whose patched quadrant currently holds
        classes ``cur``: integer draws only, the same rejection sampling from ``self.rng`` in the same order."""
        tg = _targets(self.base_dataset)
        tg_np = self.__dict__.get("_tg_np")
        if tg_np is None:
            tg_np = self._tg_np = tg.cpu().numpy() if isinstance(tg, torch.Tensor) else np.asarray(tg)
        n = len(self.base_dataset)
        integers = self.rng.integers
        js = np.empty(len(cur), dtype=np.int64)
        for i, c in enumerate(cur.tolist()):
            while True:
                j = int(integers(0, n))
                if tg_np[j] != c:
                    js[i] = j
                    break
        return js

    def apply_patch_digits(self, x: torch.Tensor, intermediate_vars: torch.Tensor, hl_node: HLNode, js):
        """Patch quadrant-of-``hl_node`` of every image of ``x`` with base-dataset digits ``js`` (device gather + one
        slice write); returns ``(x', labels' [B], ivs' [B,4])``."""
        idx, k = self.get_idx_and_intermediate(hl_node)
        dev = x.device
        data, tgd, _, cmap = self._device_state(dev)
        jt = js.to(dev) if isinstance(js, torch.Tensor) else torch.from_numpy(js).to(dev)
        digits = data[jt].float() / 255.0  # [B, s, s]
        if self.pad_size > 0:
            digits = torch.nn.functional.pad(digits, (self.pad_size,) * 4)
        out = x.clone()
        region = out[(slice(None),) + tuple(idx.as_index)]  # [B, 3, h, w] view of the patched quadrant
        region.copy_(digits.unsqueeze(1).expand_as(region))
        iv = intermediate_vars.clone()
        iv[:, k] = tgd[jt].to(iv.dtype)
        y = iv.gather(1, cmap[iv[:, 0]].unsqueeze(1).to(torch.long)).squeeze(1)
        return out, y, iv

    def patch_batch_at_hl(self, batch, intermediate_vars, hl_node: HLNode, _labels=None):
        idx, k = self.get_idx_and_intermediate(hl_node)
        new_batch, new_labels, new_ivs = [], [], []
        for i in range(len(batch)):
            x, iv, y = self.patch_at_hl_idx(batch[i], intermediate_vars[i], idx, k)
            new_batch.append(x)
            new_ivs.append(iv)
            new_labels.append(y)
        return new_batch, new_labels, new_ivs

    @staticmethod
    def concatenate_2x2(images):
        """Four PIL images -> one 2x2 RGB PIL image (reference helper)."""
        from PIL import Image
        assert len(images) == 4, "Need exactly four images"
        w, h = images[0].size
        out = Image.new("RGB", (w * 2, h * 2))
        for k, (ox, oy) in enumerate(((0, 0), (w, 0), (0, h), (w, h))):
            out.paste(images[k], (ox, oy))
        return out
