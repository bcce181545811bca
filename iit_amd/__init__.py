"""iit_amd: an MI355X-native Interchange Intervention Training (IIT) framework.

Same capabilities and API surface as tkwa/iit (model pairs, correspondences,
node_picker, IIT/behaviour/strict training, causal-effect / probe / leakiness
evaluation, reference checkpoint layout), built on a native hooked-transformer
engine with hand-written gfx950 HIP kernels, plan-driven in-kernel
interventions and RCCL data parallelism.  ``import iit`` exposes the reference
module paths on top of this package.
"""
__version__ = "0.1.0"

from .config import DEVICE, WANDB_ENTITY  # noqa: F401
from .core import *  # noqa: F401,F403
