"""MNIST-PVR <-> ResNet-18 on the MI355X (VERDICT r2 missing #1): the reference's second training workload
(/root/reference/train.py:5-23, /root/reference/iit/tasks/mnist_pvr/pvr_hl.py:68-134) through the plan-driven
wrapper (capture only the conv hook, fused quadrant / channel splice) and graph-captured phases."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _pair(mode="q", n=512, engine="native"):
    from iit_amd.model_pairs import IITBehaviorModelPair
    from iit_amd.tasks.task_loader import get_alignment, get_dataset
    torch.manual_seed(0)
    tr, te = get_dataset("mnist_pvr", {"train_size": n, "test_size": 256, "device": "cuda"})
    ll, hl, corr = get_alignment("mnist_pvr", {"input_shape": te.base_data.get_input_shape(), "device": "cuda",
                                               "mode": mode})
    pair = IITBehaviorModelPair(ll_model=ll, hl_model=hl, corr=corr,
                                training_args={"lr": 1e-3, "batch_size": 64, "early_stop": False,
                                               "lr_scheduler": None, "engine": engine})
    return pair, tr, te


@pytest.mark.parametrize("mode", ["q", "c"])
def test_native_intervention_matches_reference_hooks(mode):
    """Spatial-quadrant (``q``) and channel-quarter (``c``) splices: the plan-driven path (truncated capture of the
    one conv hook + fused splice kernel) equals the reference's run_with_cache + clone/index_put hook -- outputs and
    the gradient of every conv weight (zero gradient through the spliced slice included)."""
    pair, tr, _ = _pair(mode)
    assert pair.native()
    ll = pair.ll_model
    ll.eval()  # batch norm in inference mode: both passes see identical statistics
    base, abl = next(iter(tr.make_loader(64, 0)))
    for node in list(pair.corr.keys()):
        pair.training_args["engine"] = "native"
        ll.zero_grad(set_to_none=True)
        hl_n, ll_n = pair.do_intervention(base, abl, node)
        ll_n.float().pow(2).sum().backward()
        g_n = {k: p.grad.clone() for k, p in ll.named_parameters() if p.grad is not None}
        pair.training_args["engine"] = "reference"
        ll.zero_grad(set_to_none=True)
        hl_r, ll_r = pair.do_intervention(base, abl, node)
        ll_r.float().pow(2).sum().backward()
        g_r = {k: p.grad.clone() for k, p in ll.named_parameters() if p.grad is not None}
        assert torch.equal(hl_n, hl_r)
        assert torch.allclose(ll_n, ll_r, rtol=1e-4, atol=1e-4), (node, (ll_n - ll_r).abs().max())
        assert set(g_n) == set(g_r)
        for k in g_r:
            # MIOpen's weight-gradient convolutions may sum in a different order run to run: compare by relative norm
            err = float((g_n[k] - g_r[k]).norm() / (g_r[k].norm() + 1e-12))
            assert err < 2e-3, (node, k, err)


def test_capture_is_truncated_at_the_hook():
    """The source run stores only the conv hook (the reference caches every submodule output)."""
    pair, tr, _ = _pair()
    base, abl = next(iter(tr.make_loader(64, 0)))
    node = list(pair.corr.keys())[0]
    cache = pair.ll_source_cache(abl[0], [next(iter(pair.corr[node]))])
    assert list(cache.keys()) == ["mod.layer3.mod.1.mod.conv2.hook_point"]


def test_train_py_config_reduced_on_gpu_graphed():
    """train.py's configuration (IITBehaviorModelPair, lr 1e-3, batch 256, ReduceLROnPlateau) at reduced size on one
    MI355X: every optimizer phase runs as a captured HIP graph, metrics are finite and the model learns."""
    from iit_amd.entry import train as train_py
    pair = train_py.main(["--train-size", "4096", "--test-size", "512", "--epochs", "3"])
    g = getattr(pair, "_graph_step", None)
    assert g is not None and g.replays > 0 and not g.failed, getattr(g, "failed", None)
    d = pair.test_metrics.to_dict()
    assert all(v == v for v in d.values()), d
    assert d["val/accuracy"] > 20.0, d  # chance is 10 %
