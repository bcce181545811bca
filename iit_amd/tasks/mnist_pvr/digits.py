"""Offline MNIST stand-in: deterministic synthetic handwritten-style digits (no download).

The reference downloads MNIST at import (``/root/reference/iit/tasks/mnist_pvr/utils.py:5-6``);
this box has no network, so :class:`SyntheticMNIST` renders the ten digit glyphs
once (PIL's built-in TrueType font, thick strokes) and derives every sample by a
seeded random affine warp (rotation, scale, shear, shift) + stroke-width jitter +
noise, batched through ``grid_sample``.  It exposes the torchvision ``MNIST``
surface the PVR code uses: ``len``, ``__getitem__ -> (PIL.Image 'L' 28x28, int)``,
``.data`` (uint8 ``[N, 28, 28]``) and ``.targets`` (int64 ``[N]``).

If real MNIST idx files exist in ``$IIT_MNIST_DIR`` (``train-images-idx3-ubyte``
etc., optionally ``.gz``), :func:`load_mnist` reads them instead.
"""
from __future__ import annotations

import gzip
import os
from typing import Optional

import numpy as np
import torch

MNIST_SIZE = 28


def _glyph_templates(size: int = MNIST_SIZE) -> torch.Tensor:
    from PIL import Image, ImageDraw, ImageFont
    font = ImageFont.load_default(size=22)
    out = []
    for d in range(10):
        im = Image.new("L", (size, size), 0)
        ImageDraw.Draw(im).text((size / 2, size / 2), str(d), fill=255, font=font, anchor="mm", stroke_width=1,
                                stroke_fill=255)
        out.append(torch.from_numpy(np.array(im, dtype=np.float32) / 255.0))
    return torch.stack(out)  # [10, 28, 28]


class SyntheticMNIST(torch.utils.data.Dataset):
    def __init__(self, train: bool = True, size: Optional[int] = None, seed: int = 0):
        self.train = train
        self.size = size if size is not None else (60000 if train else 10000)
        self.seed = seed + (0 if train else 7919)
        self._data: Optional[torch.Tensor] = None
        g = torch.Generator().manual_seed(self.seed)
        self.targets = torch.randint(0, 10, (self.size,), generator=g)

    @property
    def data(self) -> torch.Tensor:
        if self._data is None:
            self._data = self._render()
        return self._data

    def _render(self, chunk: int = 8192) -> torch.Tensor:
        tmpl = _glyph_templates()
        g = torch.Generator().manual_seed(self.seed + 1)
        out = torch.empty(self.size, MNIST_SIZE, MNIST_SIZE, dtype=torch.uint8)
        for s in range(0, self.size, chunk):
            n = min(chunk, self.size - s)
            lab = self.targets[s:s + n]
            rot = (torch.rand(n, generator=g) - 0.5) * 0.6  # +-17 degrees
            scale = 0.85 + 0.3 * torch.rand(n, generator=g)
            shear = (torch.rand(n, generator=g) - 0.5) * 0.4
            shift = (torch.rand(n, 2, generator=g) - 0.5) * 0.25
            c, si = torch.cos(rot), torch.sin(rot)
            theta = torch.zeros(n, 2, 3)
            theta[:, 0, 0] = c / scale
            theta[:, 0, 1] = (-si + shear) / scale
            theta[:, 1, 0] = si / scale
            theta[:, 1, 1] = c / scale
            theta[:, :, 2] = shift
            grid = torch.nn.functional.affine_grid(theta, (n, 1, MNIST_SIZE, MNIST_SIZE), align_corners=False)
            img = torch.nn.functional.grid_sample(tmpl[lab].unsqueeze(1), grid, align_corners=False)
            thick = torch.rand(n, generator=g) < 0.35  # thicker strokes for a third of the samples
            if thick.any():
                img[thick] = torch.nn.functional.max_pool2d(img[thick], 3, stride=1, padding=1) * 0.9
            img = img.squeeze(1) + 0.05 * torch.rand(n, MNIST_SIZE, MNIST_SIZE, generator=g)
            out[s:s + n] = (img.clamp(0, 1) * 255).round().to(torch.uint8)
        return out

    def __len__(self) -> int:
        return self.size

    def __getitem__(self, i):
        from PIL import Image
        return Image.fromarray(self.data[i].numpy(), mode="L"), int(self.targets[i])


class IdxMNIST(SyntheticMNIST):
    """Real MNIST from local idx files (no download)."""

    def __init__(self, root: str, train: bool = True):
        prefix = "train" if train else "t10k"
        imgs = _read_idx(os.path.join(root, f"{prefix}-images-idx3-ubyte"))
        labels = _read_idx(os.path.join(root, f"{prefix}-labels-idx1-ubyte"))
        self.train = train
        self.size = imgs.shape[0]
        self._data = torch.from_numpy(imgs.copy())
        self.targets = torch.from_numpy(labels.astype(np.int64))


def _read_idx(path: str) -> np.ndarray:
    if not os.path.exists(path) and os.path.exists(path + ".gz"):
        path = path + ".gz"
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "rb") as f:
        raw = f.read()
    ndim = raw[3]
    dims = [int.from_bytes(raw[4 + 4 * i: 8 + 4 * i], "big") for i in range(ndim)]
    return np.frombuffer(raw, dtype=np.uint8, offset=4 + 4 * ndim).reshape(dims)


def load_mnist(train: bool = True, size: Optional[int] = None):
    root = os.environ.get("IIT_MNIST_DIR")
    if root and os.path.exists(os.path.join(root, "train-images-idx3-ubyte" + ("" if os.path.exists(
            os.path.join(root, "train-images-idx3-ubyte")) else ".gz"))):
        return IdxMNIST(root, train)
    return SyntheticMNIST(train=train, size=size)
