"""Host-side helpers of the graph phase runner (iit_amd/engine/graphs.py), on CPU."""
import torch

from iit_amd.engine.graphs import _clone_out


def test_clone_out_packs_scalars():
    """Replayed phase outputs are copied out (one stack for scalar losses) and never alias the captured buffers."""
    loss, extras = torch.tensor(1.5), {"a": torch.tensor(2.0), "b": torch.tensor(3.0)}
    l2, e2 = _clone_out((loss, extras))
    loss.fill_(0.0)
    extras["a"].fill_(0.0)
    assert float(l2) == 1.5 and float(e2["a"]) == 2.0 and float(e2["b"]) == 3.0
    v = torch.ones(3)
    _, e3 = _clone_out((torch.tensor(1.0), {"vec": v}))  # non-scalar extras: per-tensor clones
    v.zero_()
    assert float(e3["vec"].sum()) == 3.0
    t = torch.tensor(4.0)
    t2 = _clone_out(t)
    t.zero_()
    assert float(t2) == 4.0
