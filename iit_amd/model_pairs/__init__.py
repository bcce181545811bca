"""Model pairs (parity: ``/root/reference/iit/model_pairs/__init__.py:1-10``)."""
from ..core.nodes import HLNode, LLNode
from .base_model_pair import BaseModelPair
from .iit_model_pair import IITModelPair
from .iit_behavior_model_pair import IITBehaviorModelPair
from .strict_iit_model_pair import StrictIITModelPair
from .freeze_model_pair import FreezedModelPair
from .stop_grad_pair import StopGradHookedModel, StopGradModelPair
from .ioi_model_pair import IOI_ModelPair
from .probed_sequential_pair import IITProbeSequentialPair

__all__ = ["HLNode", "LLNode", "BaseModelPair", "IITModelPair", "IITBehaviorModelPair", "StrictIITModelPair",
           "FreezedModelPair", "StopGradHookedModel", "StopGradModelPair", "IOI_ModelPair",
           "IITProbeSequentialPair"]
