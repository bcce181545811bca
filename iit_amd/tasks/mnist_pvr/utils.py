"""PVR constants and the (lazily built) MNIST splits (parity: ``/root/reference/iit/tasks/mnist_pvr/utils.py``).

``mnist_train`` / ``mnist_test`` are built on first access (the reference downloads
at import); see :mod:`.digits` for the offline data source.
"""
from __future__ import annotations

from .digits import MNIST_SIZE, load_mnist

mnist_size = MNIST_SIZE

MNIST_CLASS_MAP = {k: [1, 1, 1, 1, 2, 2, 2, 3, 3, 3][k] for k in range(10)}

_SPLITS = {}


def __getattr__(name):
    if name in ("mnist_train", "mnist_test"):
        if name not in _SPLITS:
            _SPLITS[name] = load_mnist(train=name == "mnist_train")
        return _SPLITS[name]
    raise AttributeError(name)


def _to_pil(image):
    import numpy as np
    from PIL import Image
    arr = (image.detach().float().clamp(0, 1).cpu().numpy() * 255).astype(np.uint8)
    if arr.ndim == 3:
        arr = arr.transpose(1, 2, 0)
        if arr.shape[2] == 1:
            arr = arr[:, :, 0]
    return Image.fromarray(arr)


def visualize_datapoint(dataset, index, path: str = None):
    image, label, intermediate_vars = dataset[index]
    print(f"Label: {label}")
    print(f"Intermediate vars: {intermediate_vars}")
    print(f"Image shape: {image.shape}")
    visualize_image(image, path)


def visualize_image(input, path: str = None):
    im = _to_pil(input)
    if path:
        im.save(path)
    else:  # headless boxes: show() would fail
        im.save("pvr_image.png")
