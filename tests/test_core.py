"""T0: core primitives re-expressing the reference tests plus Q-decisions."""
import numpy as np
import pytest
import torch

from iit_amd.core.correspondence import Correspondence
from iit_amd.core.index import Ix, TorchIndex
from iit_amd.core.metric import MetricStore, MetricStoreCollection, MetricType, PerTokenMetricStore
from iit_amd.core.nodes import HLNode, LLNode


# ---- tests/test_index.py ---------------------------------------------------------------
def test_index_equals():
    assert Ix[:, :, :, :] == Ix[:, :, :, :]
    assert Ix[:, :, 0, :] == Ix[:, :, 0, :]
    assert Ix[:, :, 0, :] != Ix[:, :, 1, :]
    assert Ix[:, :] != Ix[:, :, 1, :]


def test_index_hash():
    assert hash(Ix[:, :, :, :]) == hash(Ix[:, :, :, :])
    assert hash(Ix[:, :, 0, :]) == hash(Ix[:, :, 0, :])
    assert hash(Ix[:, :, 0, :]) != hash(Ix[:, :, 1, :])


def test_index_intersect():
    assert Ix[:, :, :, :].intersects(Ix[:, :, :, :])
    assert Ix[:, :, :, :].intersects(Ix[:, :, 0, :])
    assert not Ix[:, :, 0, :].intersects(Ix[:, :, 2:3, :])
    assert not Ix[:, :, 2, :].intersects(Ix[:, :, 1, :])
    i1, i2 = Ix[:, :, 1, :], Ix[:, :, :, :]
    assert i1.intersects(i2)
    assert i1 == Ix[:, :, 1, :] and i2 == Ix[:, :, :, :]
    with pytest.raises(ValueError):
        Ix[:, :, 1].intersects(Ix[:, :, :, :])


def test_index_q14_fixes():
    # mixed open/closed slices (reference raised TypeError on max(None, int))
    assert Ix[:, :3].intersects(Ix[:, 2:])
    assert not Ix[:, :2].intersects(Ix[:, 2:])
    assert Ix[:, [1, 4]].intersects(Ix[:, 3:5])
    assert Ix[:, :, 2].graphviz_index() == "[:, :, 2]"
    assert repr(Ix[[None]]) == "[:]"
    assert Ix[:, 1] != "not an index"


def test_index_as_index_usable():
    t = torch.arange(24).view(2, 3, 4)
    assert torch.equal(t[Ix[:, 1, :].as_index], t[:, 1, :])
    assert torch.equal(t[Ix[[None]].as_index], t)


# ---- tests/test_corr.py ----------------------------------------------------------------
def test_correspondence():
    corr = Correspondence()
    hl = HLNode("hl", -1)
    ll = LLNode("ll", None)
    corr[hl] = ll
    assert corr[hl] == ll
    assert corr.get_suffixes() == {"attn": "attn.hook_result", "mlp": "mlp.hook_post"}
    assert type(corr[hl]) == LLNode
    assert corr["hl"] == ll  # HLNode == str
    with pytest.raises(TypeError):
        corr[hl] = {"not an LLNode"}


def test_make_corr_from_dict_and_suffixes():
    d = {"a": ["blocks.0.attn.hook_z", "blocks.1.mlp.hook_post"]}
    corr = Correspondence.make_corr_from_dict(d)  # Q13: default suffixes instead of assert
    assert corr.get_suffixes()["mlp"] == "mlp.hook_post"
    corr2 = Correspondence.make_corr_from_dict(d, make_suffixes_from_corr=True)
    assert corr2.get_suffixes() == {"attn": "attn.hook_z", "mlp": "mlp.hook_post"}
    assert corr2.to_name_dict() == {"a": sorted(d["a"])}


def test_suffix_maker():
    """Reference test_suffix_maker (Q12: it called an undefined free function)."""
    attns = [f"blocks.{i}.hook_attn_out" for i in range(6)]
    mlps = [f"blocks.{i}.mlp.hook_post" for i in range(6)]
    mk = lambda d: {HLNode(k, -1): {LLNode(n, None) for n in v} for k, v in d.items()}  # noqa: E731
    assert Correspondence.get_hook_suffix(mk({"all": [*mlps[:2], *attns[:4]]})) == {
        "attn": "hook_attn_out", "mlp": "mlp.hook_post"}
    attns = [f"blocks.{i}.attn.hook_result" for i in range(6)]
    assert Correspondence.get_hook_suffix(mk({"all": [mlps[3], attns[0]]})) == {
        "attn": "attn.hook_result", "mlp": "mlp.hook_post"}


def test_nodes():
    assert HLNode("x", 3) == "x" and hash(HLNode("x", 3)) == hash("x")
    assert LLNode("a", None).index == Ix[[None]]
    assert LLNode("a", Ix[:, 1]) == LLNode("a", Ix[:, 1])
    assert LLNode("a", Ix[:, 1]) != LLNode("a", Ix[:, 2])
    assert len({LLNode("a", Ix[:, 1]), LLNode("a", Ix[:, 1])}) == 1


# ---- tests/test_metric_logger.py -------------------------------------------------------
def test_metric_collection():
    mc = MetricStoreCollection([MetricStore("acc", MetricType.ACCURACY), MetricStore("loss", MetricType.LOSS)])
    mc.create_metric_store("new_acc", MetricType.ACCURACY)
    mc.update({"acc": 0.5, "loss": 0.2, "new_acc": 0.6})
    mc.update({"acc": 0.7, "loss": 0.1, "new_acc": 0.8})
    assert [str(m) for m in mc.metrics] == ["acc: 60.00%", "loss: 0.1500", "new_acc: 70.00%"]
    assert mc.metrics[0].get_value() == pytest.approx(((0.5 + 0.7) / 2) * 100)
    assert mc.metrics[1].get_value() == pytest.approx((0.2 + 0.1) / 2)
    with pytest.raises(AssertionError):
        mc.update({"missing": 1.0})


def test_metric_device_tensors_deferred():
    mc = MetricStoreCollection([MetricStore("acc", MetricType.ACCURACY), PerTokenMetricStore("tok")])
    mc.update({"acc": torch.tensor(0.5), "tok": torch.tensor([1.0, 0.0])})
    mc.update({"acc": torch.tensor(1.0), "tok": torch.tensor([0.0, 0.0])})
    assert mc.metrics[0].get_value() == pytest.approx(75.0)
    assert np.allclose(mc.metrics[1].get_value(), [0.5, 0.0])


def test_early_stop():
    """Q1: early stop needs every ACCURACY metric >= 100 (the reference's own test expected 99.1 to stop)."""
    from iit_amd.model_pairs import IITModelPair
    mc = MetricStoreCollection([MetricStore("acc", MetricType.ACCURACY), MetricStore("loss", MetricType.LOSS)])
    mc.create_metric_store("new_acc", MetricType.ACCURACY)
    mc.update({"acc": 0.5, "loss": 0.2, "new_acc": 0.6})
    assert IITModelPair._check_early_stop_condition(mc.metrics) is False
    mc2 = MetricStoreCollection([MetricStore("acc", MetricType.ACCURACY), MetricStore("new_acc", MetricType.ACCURACY)])
    mc2.update({"acc": 0.991, "new_acc": 0.991})
    assert IITModelPair._check_early_stop_condition(mc2.metrics) is False
    mc3 = MetricStoreCollection([MetricStore("acc", MetricType.ACCURACY), MetricStore("new_acc", MetricType.ACCURACY)])
    mc3.update({"acc": 1.0, "new_acc": 1.0})
    assert IITModelPair._check_early_stop_condition(mc3.metrics) is True


def test_IOI_early_stop():
    from iit_amd.model_pairs import IOI_ModelPair
    per_token = [1.0, 1.0, 0.005, 0.985, 0.022, 0.019, 1.0, 1.0, 0.361, 1.0, 0.084, 0.688, 1.0, 0.332, 1.0, 1.0]
    mc = IOI_ModelPair.make_test_metrics()
    mc.update({"val/iit_loss": 0.2, "val/IIA": 100, "val/accuracy": 60, "val/per_token_accuracy": per_token})
    assert IOI_ModelPair._check_early_stop_fn(mc.metrics, non_ioi_thresh=0.9) is False
    assert IOI_ModelPair._check_early_stop_fn(mc.metrics, non_ioi_thresh=0.5) is True


def test_logging_dict(tmp_path):
    from iit_amd.core.logger import LoggingDict
    ld = LoggingDict(log_dir=str(tmp_path))
    ld["a"] = 1
    ld["a"] = 1
    ld["a"] = torch.tensor([1, 2])
    text = open(ld._log_filename).read()
    assert "initial value: 1" in text and "changed from 1" in text
