"""Metric sinks: wandb when installed, else a local JSONL file.

The reference logs to wandb ``project="iit", entity=WANDB_ENTITY`` with one
``wandb.log`` per metric (``/root/reference/iit/model_pairs/base_model_pair.py:238-245,320-325``).
wandb is not installed on this image, so ``use_wandb=True`` falls back to
``runs/<timestamp>/metrics.jsonl`` with a warning instead of crashing.
"""
from __future__ import annotations

import json
import os
import time
from typing import Any, Dict, Optional


class JsonlSink:
    def __init__(self, path: str, config: Optional[Dict[str, Any]] = None):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        self.path = path
        self._f = open(path, "a")
        if config:
            self.log({"config": config})

    def log(self, record: Dict[str, Any]):
        self._f.write(json.dumps({"t": time.time(), **record}, default=str) + "\n")
        self._f.flush()

    def close(self):
        self._f.close()


class WandbSink:
    def __init__(self, project: str, entity: str, config: Optional[Dict[str, Any]] = None):
        import wandb  # noqa: F401

        self.wandb = wandb
        if not wandb.run:
            wandb.init(project=project, entity=entity)
        if config:
            wandb.config.update(config)

    def log(self, record: Dict[str, Any]):
        self.wandb.log(record)

    def close(self):
        pass


def make_sink(enabled: bool, project: str = "iit", entity: str = "", config=None, run_dir: Optional[str] = None):
    if not enabled:
        return None
    try:
        return WandbSink(project, entity, config)
    except ImportError:
        run_dir = run_dir or os.path.join("runs", time.strftime("%Y%m%d-%H%M%S"))
        print(f"WARNING: wandb not installed; logging metrics to {run_dir}/metrics.jsonl")
        return JsonlSink(os.path.join(run_dir, "metrics.jsonl"), config)
