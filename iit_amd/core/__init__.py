from .index import EVERYTHING, Index, Ix, TorchIndex
from .nodes import HLCache, HLNode, HookName, LLNode
from .correspondence import DEFAULT_SUFFIXES, Correspondence
from .metric import MetricStore, MetricStoreCollection, MetricType, PerTokenMetricStore
from .logger import LoggingDict
