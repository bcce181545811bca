"""T4: checkpoint layout round trip + bit-exact resume after an injected failure."""
import json
import os

import pytest
import torch

from iit_amd.data.iit_dataset import IITDataset, train_test_split
from iit_amd.tasks.ioi import make_ioi_corr, make_ioi_dataset_and_hl
from iit_amd.utils import checkpoint as ck


def _pair():
    from iit_amd.model_pairs import IOI_ModelPair
    from iit_amd.models.config import gpt2_config_dict
    from iit_amd.models.transformer import HookedTransformer
    cfg = gpt2_config_dict()
    cfg.update(n_layers=2, d_model=16, n_heads=2, d_head=8, d_mlp=32, device="cpu")
    torch.manual_seed(0)
    ll = HookedTransformer(cfg)
    ds, hl = make_ioi_dataset_and_hl(128, ll, device="cpu")
    pair = IOI_ModelPair(hl, ll, make_ioi_corr(2), training_args={"batch_size": 32, "lr": 1e-3, "lr_scheduler": None,
                                                                   "early_stop": False, "strict_weight": 0.4})
    tr, te = train_test_split(ds, 0.25, 42)
    return pair, IITDataset(tr, tr, seed=0, device="cpu"), IITDataset(te, te, seed=0, device="cpu")


def test_reference_layout_round_trip(tmp_path):
    pair, tr, te = _pair()
    pair.train(tr, te, epochs=1)
    d = ck.model_dir(pair, root=str(tmp_path / "models" / "ioi"))
    assert d.endswith(os.path.join("IOI_ModelPair", "100_100_40"))
    ck.save_reference_layout(d, pair, epochs=1)
    for f in ("ll_model.pth", "training_args.json", "ll_model_cfg.json", "metrics.log", "corr.json"):
        assert os.path.exists(os.path.join(d, f)), f
    sd = torch.load(os.path.join(d, "ll_model.pth"), weights_only=True)
    assert "blocks.0.attn.W_Q" in sd and sd["blocks.0.attn.W_Q"].is_contiguous()
    args = json.load(open(os.path.join(d, "training_args.json")))
    assert args["strict_weight"] == 0.4
    corr = json.load(open(os.path.join(d, "corr.json")))
    assert corr["hook_duplicate"] == ["blocks.0.attn.hook_z"]
    assert "val/IIA" in open(os.path.join(d, "metrics.log")).read()
    fresh, _, _ = _pair()
    ck.load_ll_model(d, fresh.ll_model)
    for (n, a), (_, b) in zip(pair.ll_model.named_parameters(), fresh.ll_model.named_parameters()):
        assert torch.equal(a, b), n
    c2 = ck.load_corr(d, suffixes=pair.corr.get_suffixes())
    assert set(k.name for k in c2.keys()) == set(k.name for k in pair.corr.keys())


class _Crash(RuntimeError):
    pass


def test_resume_after_injected_failure_is_bit_exact(tmp_path):
    ref, tr, te = _pair()
    ref.train(tr, te, epochs=3)

    run, tr2, te2 = _pair()

    def kill_after_first_epoch(epoch):
        if epoch == 0:
            raise _Crash("injected rank failure")

    with pytest.raises(_Crash):
        run.train(tr2, te2, epochs=3, checkpoint_dir=str(tmp_path / "ckpt"), fault_hook=kill_after_first_epoch)
    assert ck.has_resume_state(str(tmp_path / "ckpt"))

    resumed, tr3, te3 = _pair()  # a fresh process: new model, new RNG streams
    torch.manual_seed(1234)
    resumed.rng.random()  # perturb the node-sampling generator: resume must restore it
    resumed.train(tr3, te3, epochs=3, checkpoint_dir=str(tmp_path / "ckpt"), resume=True)
    for (n, a), (_, b) in zip(ref.ll_model.named_parameters(), resumed.ll_model.named_parameters()):
        assert torch.equal(a, b), n
