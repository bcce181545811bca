"""Utilities (parity surface of ``/root/reference/iit/utils/__init__.py:1-4``)."""
from ..config import DEVICE, WANDB_ENTITY
from ..core.index import Ix
from ..data.iit_dataset import IITDataset
from ..hooks.wrapper import HookedModuleWrapper
