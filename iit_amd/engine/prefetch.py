"""Double-buffered source-activation caches (BASELINE.json north star: "source-activation caches are
double-buffered in 288 GB HBM per GPU").

An interchange intervention needs the LL model's activations on the *source* input before the spliced *base*
forward can run.  Within one optimizer step nothing can be overlapped (the base forward consumes the cache, and
the next step's source run needs the updated weights), but wherever the weights are fixed -- evaluation epochs,
causal-effect sweeps -- the source forward of batch k+1 does not depend on batch k at all.
:class:`SourcePrefetcher` runs it early, on a side HIP stream, into the other of two cache slots:

    compute stream:  [base k-1 + HL + metrics] [base k + HL + metrics] [base k+1 ...
    side stream:       [source k]                [source k+1]             [source k+2] ...

The HL node of batch k+1 is drawn from the pair's RNG when its prefetch launches (in batch order: the serial
sequence), so each slot holds exactly the LL sites of that node, captured by the same truncated source forward.  The compute stream waits
on the slot's event before reading it, the tensors are marked as used by the compute stream
(``record_stream``), and a slot is only overwritten two batches later.  The captured values are identical to the
pair's own (truncated) source run: same kernels, same inputs, the same weights.

Measured on one MI355X (``scripts/bench_eval.py``, 12,000 IOI pairs, batch 512): GPT-2-small eval 38.6k pairs/s
serial vs 37.0-38.9k prefetched, the 6L/64d reference model 97.7k vs 91.2-95.0k -- no gain: the GPT-2 epoch is
GPU-bound (two streams of large GEMMs do not run faster than one on this chip, see scripts/diag_concurrency.py)
and the small model's is host-bound (prefetching moves, not removes, launch work).  It is therefore opt-in
(``training_args['prefetch_source'] = True``).
"""
from __future__ import annotations

from typing import Dict, Iterable, Optional

import torch


class SourcePrefetcher:
    def __init__(self, pair, names: Optional[Iterable[str]] = None):
        from ..model_pairs.base_model_pair import _ll_nodes_of
        self.pair = pair
        if names is None:
            names = {n.name for hl in pair.corr for n in _ll_nodes_of(pair.corr, hl)}
        self.names = sorted(names)
        self.stream = torch.cuda.Stream()
        self.slots = [None, None]
        self.hits = 0

    def launch(self, slot: int, x: torch.Tensor) -> None:
        """Start the source forward of ``x`` on the side stream into cache slot ``slot``."""
        main = torch.cuda.current_stream()
        self.stream.wait_stream(main)  # x (and the previous slot's readers) were enqueued on the compute stream
        with torch.cuda.stream(self.stream):
            caps = self.pair.ll_model.run_capture(x, self.names)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        x.record_stream(self.stream)
        self.slots[slot] = (x, caps, ev)

    def lookup(self, x: torch.Tensor, names: Iterable[str]) -> Optional[Dict[str, torch.Tensor]]:
        """The prefetched activations ``names`` of source input ``x`` (None when ``x`` was not prefetched)."""
        for ent in self.slots:
            if ent is None or ent[0] is not x:
                continue
            _, caps, ev = ent
            names = list(names)
            if not all(n in caps for n in names):
                return None
            cur = torch.cuda.current_stream()
            cur.wait_event(ev)
            out = {}
            for n in names:
                caps[n].record_stream(cur)
                out[n] = caps[n]
            self.hits += 1
            return out
        return None


def supported(pair) -> bool:
    """Prefetch applies to native LL engines on the GPU (opt-in: ``training_args['prefetch_source']``)."""
    if not torch.cuda.is_available() or not pair.training_args.get("prefetch_source", False):
        return False
    try:
        dev = next(pair._ll_module().parameters()).device
    except StopIteration:
        return False
    return dev.type == "cuda" and pair.native() and hasattr(pair.ll_model, "run_capture")


def prefetched_batches(pair, loader):
    """Iterate ``loader``'s (base, source) batches while the next batch's source forward runs ahead.

    Every eval step draws exactly one HL node (``sample_hl_name``) first; the node of batch k+1 is drawn when
    its prefetch is launched (still in batch order, so the RNG sequence is the serial one) and handed to the
    step through a queue, so the side stream captures only that node's LL sites and stops at the deepest of
    them -- the same truncated source forward the serial step would run.  The prefetcher is installed on the
    pair for the duration (``ll_source_cache`` consults it)."""
    from ..model_pairs.base_model_pair import _ll_nodes_of
    pf = SourcePrefetcher(pair)
    queue = []
    orig = pair.__dict__.get("sample_hl_name")
    draw = pair.sample_hl_name

    def launch(slot, batch):
        node = draw()
        queue.append(node)
        pf.names = sorted({n.name for n in _ll_nodes_of(pair.corr, node)})
        pf.launch(slot, batch[1][0])

    pair._source_prefetch = pf
    pair.sample_hl_name = lambda: queue.pop(0)
    try:
        it = iter(loader)
        cur = next(it, None)
        k = 0
        if cur is not None:
            launch(0, cur)
        while cur is not None:
            nxt = next(it, None)
            if nxt is not None:
                launch((k + 1) % 2, nxt)
            yield cur
            cur = nxt
            k += 1
    finally:
        pair._source_prefetch = None
        if orig is None:
            pair.__dict__.pop("sample_hl_name", None)
        else:
            pair.sample_hl_name = orig
