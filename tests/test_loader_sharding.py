"""DeviceIITLoader sharding under data parallelism: epoch tails are split into balanced, never-empty
shards; a tail smaller than the world size is skipped by every rank."""
import pytest
import torch

from iit_amd.data.iit_dataset import DeviceIITLoader, IITDataset, IITUniqueDataset


class _Toy:
    """A gather-capable dataset: row i is (x=[i], y=[i], iv=[i])."""

    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        t = torch.tensor([i])
        return t, t, t

    def gather(self, idx):
        t = idx.view(-1, 1)
        return t, t, t


def _shards(n, batch, world):
    # the unpaired dataset yields x = the dataset row, so shard contents are checkable
    ds = IITUniqueDataset(_Toy(n), None, seed=0, device="cpu")
    paired = IITDataset(_Toy(n), _Toy(n), seed=0, device="cpu")
    out = []
    for rank in range(world):
        ld = DeviceIITLoader(ds, batch, shuffle=False)
        ld.rank, ld.world = rank, world
        out.append([b[0].view(-1).tolist() for b in ld])
        assert len(out[-1]) == len(ld)
        lp = DeviceIITLoader(paired, batch, shuffle=False)
        lp.rank, lp.world = rank, world
        assert [len(b[0][0]) for b in lp] == [len(b) for b in out[-1]]
    return out


@pytest.mark.parametrize("n,batch,world", [(8 * 4 + 10, 4, 8), (8 * 4 + 5, 4, 8), (8 * 4 + 8, 4, 8),
                                           (8 * 4 + 9, 4, 8), (2 * 3 + 1, 3, 2), (20, 4, 8)])
def test_tail_shards_never_empty_and_balanced(n, batch, world):
    shards = _shards(n, batch, world)
    n_batches = {len(s) for s in shards}
    assert len(n_batches) == 1  # every rank runs the same number of steps (same collective sequence)
    for step in range(len(shards[0])):
        sizes = [len(s[step]) for s in shards]
        assert min(sizes) >= 1 and max(sizes) - min(sizes) <= 1, sizes
        rows = sorted(r for s in shards for r in s[step])
        assert len(rows) == len(set(rows))  # disjoint shards
    tail = n % (batch * world)
    covered = sum(len(b) for s in shards for b in s)
    assert covered == (n if tail == 0 or tail >= world else n - tail)


def test_single_process_keeps_the_whole_tail():
    shards = _shards(10, 4, 1)
    assert [len(b) for b in shards[0]] == [4, 4, 2]
