"""MNIST pointer-value retrieval task (offline synthetic digits; see :mod:`.digits`)."""
from .dataset import ImagePVRDataset
from .get_alignment import get_alignment
from .pvr_check_leaky_hl import MNIST_PVR_Leaky_HL
from .pvr_check_leaky_hl import get_corr as get_corr_leaky
from .pvr_hl import MNIST_PVR_HL, get_corr, hl_nodes
from .utils import MNIST_CLASS_MAP, mnist_size


def __getattr__(name):
    if name in ("mnist_train", "mnist_test"):
        from . import utils
        return getattr(utils, name)
    raise AttributeError(name)
