"""(base, source) pair datasets and device-resident loaders.

Parity: ``/root/reference/iit/utils/iit_dataset.py:9-84`` and
``/root/reference/iit/utils/eval_datasets.py:7-19``.

* Item ``i`` pairs ``base_data[rng.choice(n_base)]`` with
  ``ablation_data[rng.choice(n_abl)]`` where ``rng = default_rng(seed*1e6 + i)``,
  so pairs are fixed per index and reshuffled by the loader each epoch;
  ``every_combination=True`` enumerates the cross product.
* The epoch order reproduces ``DataLoader(shuffle=True)`` bit-for-bit: the same
  two draws from the torch global RNG (``_base_seed`` then the sampler seed)
  followed by ``randperm`` on a CPU generator.

MI355X-first data path (SURVEY.md §3.1 hot loop 3): when the underlying datasets
expose ``gather(idx)`` (the synthetic IOI / PVR datasets do), ``make_loader``
returns a :class:`DeviceIITLoader` that keeps the pair table and the samples in
HBM and assembles each batch with two ``index_select`` launches - no per-sample
Python, no host->device copies.  Other datasets use a regular ``DataLoader``
with the reference collate.  Under ``torch.distributed`` each rank takes its
contiguous shard of every *global* batch (``batch_size`` is per rank).  The
epoch tail is split into balanced shards (sizes differ by at most one row); a
tail smaller than the world size is skipped, so no rank ever sees an empty batch.
"""
from __future__ import annotations

from typing import Iterator, Optional, Sequence, Tuple

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset, Subset

from ..config import DEVICE


def _gather_fn(ds):
    """Return ``f(idx_tensor) -> (x, y, iv)`` if ``ds`` supports batched gathers, else None."""
    if hasattr(ds, "gather"):
        return ds.gather
    if isinstance(ds, Subset):
        inner = _gather_fn(ds.dataset)
        if inner is None:
            return None
        table = torch.as_tensor(list(ds.indices), dtype=torch.long)
        cache = {}

        def f(idx, _inner=inner, _table=table, _cache=cache):
            dev = idx.device
            t = _cache.get(dev)
            if t is None:
                t = _cache[dev] = _table.to(dev)
            return _inner(t.index_select(0, idx))

        return f
    return None


def _dist_info() -> Tuple[int, int]:
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        return torch.distributed.get_rank(), torch.distributed.get_world_size()
    return 0, 1


def loader_epoch_permutation(n: int) -> torch.Tensor:
    """The index order ``DataLoader(shuffle=True)`` would produce for this epoch."""
    torch.empty((), dtype=torch.int64).random_()  # DataLoaderIter._base_seed
    seed = int(torch.empty((), dtype=torch.int64).random_().item())  # RandomSampler seed
    g = torch.Generator()
    g.manual_seed(seed)
    return torch.randperm(n, generator=g)


class IITDataset(Dataset):
    def __init__(self, base_data, ablation_data, seed: int = 0, every_combination: bool = False, device=DEVICE):
        self.base_data = base_data
        self.ablation_data = ablation_data
        self.seed = seed
        self.every_combination = every_combination
        self.device = device
        self._pair_table: Optional[Tuple[np.ndarray, np.ndarray]] = None

    # -- pair sampling -------------------------------------------------------------
    def pair_indices(self, index: int) -> Tuple[int, int]:
        if self.every_combination:
            n_abl = len(self.ablation_data)
            return index // n_abl, index % n_abl
        rng = np.random.default_rng(self.seed * 1000000 + index)
        base = rng.choice(len(self.base_data))
        abl = rng.choice(len(self.ablation_data))
        return int(base), int(abl)

    def pair_table(self) -> Tuple[np.ndarray, np.ndarray]:
        if self._pair_table is None:
            n = len(self)
            if self.every_combination:
                idx = np.arange(n)
                n_abl = len(self.ablation_data)
                self._pair_table = (idx // n_abl, idx % n_abl)
            else:
                pairs = np.array([self.pair_indices(i) for i in range(n)], dtype=np.int64).reshape(n, 2)
                self._pair_table = (pairs[:, 0], pairs[:, 1])
        return self._pair_table

    def __getitem__(self, index):
        b, a = self.pair_indices(index)
        return self.base_data[b], self.ablation_data[a]

    def __len__(self) -> int:
        if self.every_combination:
            return len(self.base_data) * len(self.ablation_data)
        return len(self.base_data)

    # -- collation -------------------------------------------------------------------
    @staticmethod
    def get_encoded_input_from_torch_input(xy, device=DEVICE):
        x, y, iv = zip(*xy)
        stack = lambda seq: torch.stack([torch.as_tensor(s).to(device) for s in seq])  # noqa: E731
        return stack(x), stack(y), stack(iv)

    @staticmethod
    def collate_fn(batch, device=DEVICE):
        base, abl = zip(*batch)
        return (IITDataset.get_encoded_input_from_torch_input(base, device),
                IITDataset.get_encoded_input_from_torch_input(abl, device))

    def supports_device_loader(self) -> bool:
        return _gather_fn(self.base_data) is not None and _gather_fn(self.ablation_data) is not None

    def make_loader(self, batch_size: int, num_workers: int = 0, shuffle: bool = True, fast: Optional[bool] = None):
        if fast is None:
            fast = self.supports_device_loader()
        if fast:
            return DeviceIITLoader(self, batch_size, shuffle=shuffle)
        return DataLoader(self, batch_size=batch_size, shuffle=shuffle, num_workers=num_workers,
                          collate_fn=lambda b: self.collate_fn(b, self.device))


class DeviceIITLoader:
    """HBM-resident ``(base, source)`` batch stream with reference shuffle semantics."""

    def __init__(self, dataset: IITDataset, batch_size: int, shuffle: bool = True, drop_last: bool = False,
                 device=None):
        self.dataset = dataset
        self.batch_size = batch_size
        self.shuffle = shuffle
        self.drop_last = drop_last
        self.rank, self.world = _dist_info()
        self.device = torch.device(device) if device is not None else torch.device(dataset.device)
        self._base_gather = _gather_fn(dataset.base_data)
        self._abl_gather = _gather_fn(dataset.ablation_data)
        self._unique = isinstance(dataset, IITUniqueDataset)
        self._tables = None

    def _device_tables(self):
        if self._tables is None:
            if self._unique:
                self._tables = (None, None)
            else:
                b, a = self.dataset.pair_table()
                self._tables = (torch.as_tensor(b).to(self.device), torch.as_tensor(a).to(self.device))
        return self._tables

    @property
    def global_batch(self) -> int:
        return self.batch_size * self.world

    def __len__(self) -> int:
        n = len(self.dataset)
        gb = self.global_batch
        if self.drop_last or (self.world > 1 and 0 < n % gb < self.world):
            return n // gb
        return (n + gb - 1) // gb

    def __iter__(self) -> Iterator:
        n = len(self.dataset)
        perm = loader_epoch_permutation(n) if self.shuffle else torch.arange(n)
        if self.device.type == "cuda":
            # pinned + asynchronous: a pageable copy would block the host until the GPU drained every queued step,
            # and the first launches of the next epoch then run on an idle GPU
            perm = perm.pin_memory().to(self.device, non_blocking=True)
        else:
            perm = perm.to(self.device)
        base_t, abl_t = self._device_tables()
        gb = self.global_batch
        for start in range(0, n, gb):
            chunk = perm[start:start + gb]
            if chunk.numel() < gb and self.drop_last:
                break
            if self.world > 1:
                if chunk.numel() < self.world:
                    # a tail that cannot give every rank a row: an empty shard would average NaN losses and
                    # accuracies into every rank's metrics (and trip the early stop), so all ranks skip it
                    break
                # balanced shards (sizes differ by at most one row), never empty
                chunk = torch.tensor_split(chunk, self.world)[self.rank]
            if self._unique:
                yield self._base_gather(chunk)
            else:
                yield (self._base_gather(base_t.index_select(0, chunk)),
                       self._abl_gather(abl_t.index_select(0, chunk)))


class IITUniqueDataset(IITDataset):
    """Un-paired dataset for mean / zero ablation sweeps (``eval_datasets.py:7-19``)."""

    def __getitem__(self, index):
        return self.base_data[index]

    def __len__(self) -> int:
        return len(self.base_data)

    @staticmethod
    def collate_fn(batch, device=DEVICE):
        return IITDataset.get_encoded_input_from_torch_input(batch, device)

    def supports_device_loader(self) -> bool:
        return _gather_fn(self.base_data) is not None

    def make_loader(self, batch_size: int, num_workers: int = 0, shuffle: bool = True, fast: Optional[bool] = None):
        if fast is None:
            fast = self.supports_device_loader()
        if fast:
            return DeviceIITLoader(self, batch_size, shuffle=shuffle)
        return DataLoader(self, batch_size=batch_size, shuffle=shuffle, num_workers=num_workers,
                          collate_fn=lambda b: self.collate_fn(b, self.device))


def train_test_split(dataset, test_size: float = 0.2, random_state: Optional[int] = None):
    n = len(dataset)
    split = int(n * test_size)
    if random_state is None:
        return torch.utils.data.random_split(dataset, [n - split, split])
    return torch.utils.data.random_split(dataset, [n - split, split],
                                         generator=torch.Generator().manual_seed(random_state))
