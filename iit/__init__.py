"""Reference-compatible import surface: ``import iit.model_pairs`` etc. resolve to ``iit_amd``.

A user of tkwa/iit keeps their imports (``from iit.utils.index import Ix``,
``import iit.model_pairs as mp``, ``from iit.tasks.ioi import corr``...).  Each
``iit.*`` module is created lazily by a meta-path finder and shares every object
(classes, functions, constants) with the ``iit_amd`` module that implements it.
"""
from __future__ import annotations

import importlib
import importlib.abc
import importlib.util
import sys

_ALIASES = {
    "iit.model_pairs": "iit_amd.model_pairs",
    "iit.model_pairs.base_model_pair": "iit_amd.model_pairs.base_model_pair",
    "iit.model_pairs.iit_model_pair": "iit_amd.model_pairs.iit_model_pair",
    "iit.model_pairs.iit_behavior_model_pair": "iit_amd.model_pairs.iit_behavior_model_pair",
    "iit.model_pairs.strict_iit_model_pair": "iit_amd.model_pairs.strict_iit_model_pair",
    "iit.model_pairs.freeze_model_pair": "iit_amd.model_pairs.freeze_model_pair",
    "iit.model_pairs.stop_grad_pair": "iit_amd.model_pairs.stop_grad_pair",
    "iit.model_pairs.ioi_model_pair": "iit_amd.model_pairs.ioi_model_pair",
    "iit.model_pairs.probed_sequential_pair": "iit_amd.model_pairs.probed_sequential_pair",
    "iit.model_pairs.nodes": "iit_amd.core.nodes",
    "iit.utils": "iit_amd.utils",
    "iit.utils.index": "iit_amd.core.index",
    "iit.utils.correspondence": "iit_amd.core.correspondence",
    "iit.utils.metric": "iit_amd.core.metric",
    "iit.utils.logger": "iit_amd.core.logger",
    "iit.utils.config": "iit_amd.config",
    "iit.utils.iit_dataset": "iit_amd.data.iit_dataset",
    "iit.utils.eval_datasets": "iit_amd.data.iit_dataset",
    "iit.utils.node_picker": "iit_amd.utils.node_picker",
    "iit.utils.eval_ablations": "iit_amd.utils.eval_ablations",
    "iit.utils.eval_metrics": "iit_amd.utils.eval_metrics",
    "iit.utils.probes": "iit_amd.utils.probes",
    "iit.utils.plotter": "iit_amd.utils.plotter",
    "iit.utils.wrapper": "iit_amd.hooks.wrapper",
    "iit.tasks": "iit_amd.tasks",
    "iit.tasks.hl_model": "iit_amd.tasks.hl_model",
    "iit.tasks.task_loader": "iit_amd.tasks.task_loader",
    "iit.tasks.ioi": "iit_amd.tasks.ioi",
    "iit.tasks.ioi.ioi_hl": "iit_amd.tasks.ioi.ioi_hl",
    "iit.tasks.ioi.ioi_config": "iit_amd.tasks.ioi.ioi_config",
    "iit.tasks.ioi.ioi_dataset_tl": "iit_amd.tasks.ioi.ioi_dataset",
    "iit.tasks.ioi.utils": "iit_amd.tasks.ioi",
    "iit.tasks.mnist_pvr": "iit_amd.tasks.mnist_pvr",
    "iit.tasks.mnist_pvr.dataset": "iit_amd.tasks.mnist_pvr.dataset",
    "iit.tasks.mnist_pvr.pvr_hl": "iit_amd.tasks.mnist_pvr.pvr_hl",
    "iit.tasks.mnist_pvr.pvr_check_leaky_hl": "iit_amd.tasks.mnist_pvr.pvr_check_leaky_hl",
    "iit.tasks.mnist_pvr.get_alignment": "iit_amd.tasks.mnist_pvr.get_alignment",
    "iit.tasks.mnist_pvr.utils": "iit_amd.tasks.mnist_pvr.utils",
    "iit.tasks.docstring": "iit_amd.tasks.docstring",
    "iit.tasks.docstring.docstring_hl": "iit_amd.tasks.docstring.docstring_hl",
}


class _AliasLoader(importlib.abc.Loader):
    def create_module(self, spec):
        return None

    def exec_module(self, module):
        target = importlib.import_module(_ALIASES[module.__name__])
        for k, v in vars(target).items():
            if not (k.startswith("__") and k.endswith("__")):
                module.__dict__[k] = v
        module.__dict__["__all__"] = getattr(target, "__all__", [k for k in vars(target) if not k.startswith("_")])
        module.__path__ = []  # behave as a package so deeper aliases resolve


class _AliasFinder(importlib.abc.MetaPathFinder):
    def find_spec(self, fullname, path, target=None):
        if fullname in _ALIASES:
            return importlib.util.spec_from_loader(fullname, _AliasLoader(), is_package=True)
        return None


if not any(isinstance(f, _AliasFinder) for f in sys.meta_path):
    sys.meta_path.insert(0, _AliasFinder())


def __getattr__(name):
    full = f"iit.{name}"
    if full in _ALIASES:
        return importlib.import_module(full)
    raise AttributeError(name)
