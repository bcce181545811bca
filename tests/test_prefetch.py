"""Double-buffered source-activation caches (iit_amd.engine.prefetch): an evaluation epoch with the next batch's
source forward running ahead on a side stream gives exactly the metrics of the serial epoch."""
import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _pair(prefetch: bool):
    from iit_amd.data.iit_dataset import IITDataset
    from iit_amd.model_pairs import IOI_ModelPair
    from iit_amd.models.config import gpt2_config_dict
    from iit_amd.models.transformer import HookedTransformer
    from iit_amd.tasks.ioi import make_ioi_corr, make_ioi_dataset_and_hl
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    cfg = gpt2_config_dict()
    cfg.update(n_layers=6, d_model=128, n_heads=4, d_head=32, d_mlp=512, device="cuda:0", dtype=torch.bfloat16)
    ll = HookedTransformer(cfg)
    ds, hl = make_ioi_dataset_and_hl(640, ll, device=dev)
    test = IITDataset(ds, ds, seed=0, device=dev)
    pair = IOI_ModelPair(hl, ll, make_ioi_corr(6), training_args={"batch_size": 64, "lr_scheduler": None,
                                                                   "prefetch_source": prefetch})
    return pair, test


def test_prefetched_eval_epoch_equals_serial():
    from iit_amd.engine import prefetch
    a, test = _pair(True)
    b, _ = _pair(False)
    b.ll_model.load_state_dict(a.ll_model.state_dict())
    b.rng = copy.deepcopy(a.rng)
    assert prefetch.supported(a) and not prefetch.supported(b)
    calls = []
    orig = prefetch.SourcePrefetcher.lookup
    prefetch.SourcePrefetcher.lookup = lambda self, x, names: calls.append(1) or orig(self, x, names)
    try:
        torch.manual_seed(1)
        ma = a._run_eval_epoch(test.make_loader(64, 0, shuffle=False), a.loss_fn).to_dict()
    finally:
        prefetch.SourcePrefetcher.lookup = orig
    torch.manual_seed(1)
    mb = b._run_eval_epoch(test.make_loader(64, 0, shuffle=False), b.loss_fn).to_dict()
    assert len(calls) == 10  # every batch's source cache came from the prefetcher
    for k in ma:
        assert np.allclose(np.asarray(ma[k]), np.asarray(mb[k]), atol=1e-6), k
    assert getattr(a, "_source_prefetch", None) is None
