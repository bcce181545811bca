"""Tracing, step timing and the race-debug switch.

The reference has no tracing at all (``/root/reference/iit/model_pairs/base_model_pair.py:246,282``: tqdm bars only).
This module adds, behind environment switches read once at import:

* ``IIT_PROFILE=1`` -- named ranges around every phase of a training step (HL source / LL source capture / HL
  intervened / LL spliced forward, backward, gradient all-reduce, clip + Adam, graph replays, evaluation).  Each
  range is a roctx range (``torch.cuda.nvtx`` is roctx on ROCm builds: ``rocprofv3 --marker-trace`` records them
  next to the kernels) and a ``torch.profiler.record_function`` region (the torch profiler's timeline).  Off, a
  range is one attribute check.
* ``IIT_DEBUG_SYNC=1`` -- the race-debug mode: :func:`sync_point` drains the device at every phase boundary, so
  no two phases (source capture vs spliced forward, backward vs all-reduce, ...) can overlap on different streams;
  the import of :mod:`iit_amd.config` also sets ``HIP_LAUNCH_BLOCKING=1`` / ``AMD_SERIALIZE_KERNEL=3`` (kernel
  launches serialised by the runtime) unless they are already set.

:class:`StepTimer` times training steps with HIP events (no host sync per step; resolved once per epoch) and
reports ms/step and intervened (base, source) pairs/s -- whole-job, over data-parallel ranks.
"""
from __future__ import annotations

import contextlib
import time
from typing import Dict, List, Optional

import torch

from ..config import debug_sync, profiling_enabled

PROFILE = profiling_enabled()
DEBUG_SYNC = debug_sync()


class _Range:
    """roctx + torch-profiler range (entered only when profiling is on)."""
    __slots__ = ("name", "_rf", "_nvtx")

    def __init__(self, name: str):
        self.name = name
        self._rf = None
        self._nvtx = False

    def __enter__(self):
        if torch.cuda.is_available():
            try:
                torch.cuda.nvtx.range_push(self.name)
                self._nvtx = True
            except Exception:  # noqa: BLE001 - a build without roctx: the torch-profiler region still records
                self._nvtx = False
        self._rf = torch.profiler.record_function(self.name)
        self._rf.__enter__()
        return self

    def __exit__(self, *exc):
        self._rf.__exit__(*exc)
        if self._nvtx:
            torch.cuda.nvtx.range_pop()
        return False


_NULL = contextlib.nullcontext()


def trace_range(name: str):
    """Context manager: a named range when ``IIT_PROFILE=1`` (or :func:`set_profiling`), else a no-op."""
    return _Range(name) if PROFILE else _NULL


def set_profiling(on: bool) -> None:
    """Turn the ranges on / off at run time (tests, notebooks); the environment sets the initial state."""
    global PROFILE
    PROFILE = bool(on)


def set_debug_sync(on: bool) -> None:
    global DEBUG_SYNC
    DEBUG_SYNC = bool(on)


def sync_point() -> None:
    """Phase boundary: in race-debug mode (``IIT_DEBUG_SYNC=1``) wait for all device work, so phases on different
    streams never overlap; otherwise nothing.  Inside a graph capture it does nothing (a device sync would abort
    the capture; the captured phases replay in stream order anyway)."""
    if DEBUG_SYNC and torch.cuda.is_available() and not torch.cuda.is_current_stream_capturing():
        torch.cuda.synchronize()


class StepTimer:
    """Per-step device time of a training epoch from HIP events recorded on the current stream (host clock off
    the GPU).  ``start()`` / ``stop(pairs)`` bracket one step; ``summary()`` (once per epoch) resolves the events
    and returns ms/step and whole-job pairs/s (the per-rank batch times ``world_size``).  Steps whose batch has a
    different size (the epoch tail) are timed like the others and counted with their own pair count."""

    def __init__(self, world_size: int = 1):
        self.world = max(1, int(world_size))
        self.cuda = torch.cuda.is_available()
        self._marks: List[tuple] = []
        self._open = None

    def start(self) -> None:
        if self.cuda:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self._open = ev
        else:
            self._open = time.perf_counter()

    def stop(self, pairs: int) -> None:
        if self._open is None:
            return
        if self.cuda:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self._marks.append((self._open, ev, int(pairs)))
        else:
            self._marks.append((self._open, time.perf_counter(), int(pairs)))
        self._open = None

    def summary(self, skip_first: int = 1) -> Optional[Dict[str, float]]:
        """{"ms_per_step", "pairs_per_s", "steps"} over the epoch's steps after the first ``skip_first`` (warm-up,
        graph capture), or over all of them when there are no others; None when no step was timed."""
        marks = self._marks
        self._marks = []
        if not marks:
            return None
        if len(marks) > skip_first:
            marks = marks[skip_first:]
        if self.cuda:
            marks[-1][1].synchronize()
            ms = [a.elapsed_time(b) for a, b, _ in marks]
        else:
            ms = [(b - a) * 1e3 for a, b, _ in marks]
        total_ms = sum(ms)
        pairs = sum(p for _, _, p in marks) * self.world
        return {"ms_per_step": total_ms / len(ms), "pairs_per_s": pairs / (total_ms / 1e3) if total_ms > 0 else 0.0,
                "steps": float(len(ms))}
