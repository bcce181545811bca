"""The restructured PVR leakiness sweep (entry/eval_causality.py ``_fast_resample_sweep``: twelve HL nodes per
launch sequence, truncated source runs, base prefix shared and spliced runs started at the hook) against the
per-node path (one ``do_intervention`` per (hook point, batch, node), the reference loop) on the same patch draws."""
import numpy as np
import pytest
import torch


def _setup(test_size, seed=0):
    from iit_amd.tasks.task_loader import get_alignment, get_dataset
    torch.manual_seed(seed)
    _, leaky = get_dataset("pvr_leaky", dataset_config={"train_size": 1, "test_size": test_size, "device": "cpu"})
    ll, _, _ = get_alignment("mnist_pvr", config={"input_shape": leaky.base_data.get_input_shape(), "device": "cpu"})
    ll.eval()
    return ll, leaky.base_data


@pytest.mark.parametrize("hooks", [("mod.conv1.hook_point", "mod.layer1.mod.0.mod.conv2.hook_point"),
                                   ("mod.layer2.mod.0.mod.conv1.hook_point", "mod.layer3.mod.1.mod.conv2.hook_point",
                                    "mod.layer4.mod.1.mod.conv1.hook_point")])
def test_fast_sweep_equals_per_node_path(hooks):
    from iit_amd.entry.eval_causality import evaluate_model_on_ablations
    ll, ds_a = _setup(48)
    _, ds_b = _setup(48)
    fast = evaluate_model_on_ablations(ll, "pvr_leaky", ds_a, {"batch_size": 20}, hook_points=list(hooks))
    slow = evaluate_model_on_ablations(ll, "pvr_leaky", ds_b, {"batch_size": 20, "fast": False},
                                       hook_points=list(hooks))
    assert ds_a.rng.bit_generator.state == ds_b.rng.bit_generator.state  # the same draws, in the same order
    for h in hooks:
        assert set(fast[h]) == set(slow[h]) and len(fast[h]) == 12
        a = np.array([fast[h][k] for k in sorted(fast[h])])
        b = np.array([slow[h][k] for k in sorted(fast[h])])
        assert np.abs(a - b).max() <= 1e-6, (h, a, b)


def test_hl_output_is_the_patched_label():
    """The fast sweep takes the HL output of hook_{i}_leaked_to_{j} from the patched batch's label."""
    from iit_amd.model_pairs import IITProbeSequentialPair
    from iit_amd.tasks.task_loader import get_alignment
    ll, ds = _setup(32)
    x, y, iv = ds.gather(torch.arange(0, 32))
    _, hl, corr = get_alignment("pvr_leaky", config={"hook_point": "mod.layer1.mod.0.mod.conv1.hook_point",
                                                     "input_shape": ds.get_input_shape(), "device": "cpu"})
    pair = IITProbeSequentialPair(ll_model=ll, hl_model=hl, corr=corr)
    for nd in pair.corr:
        _, k = ds.get_idx_and_intermediate(nd)
        js = ds.draw_patch_digits(iv[:, k].numpy())
        ab = ds.apply_patch_digits(x, iv, nd, js)
        hl_out, _ = pair.do_intervention((x, y, iv), ab, nd)
        assert torch.equal(hl_out.long(), ab[1].long()), nd.name


def test_cached_probe_evaluation_equals_per_probe_loop():
    """The native engine's probe sweep (utils/probes.py ActivationBank: every hook point's train / test activations
    captured once, probes trained and evaluated from gathers) equals the reference engine's path (one capture per
    hook point and batch for training, one per probe and batch for evaluation) on the same shuffle draws."""
    from torch import nn

    from iit_amd.entry.eval_information import evaluate_model_on_probes
    from iit_amd.tasks.task_loader import get_dataset
    ll, _ = _setup(8)
    tr, te = get_dataset("pvr_leaky", dataset_config={"train_size": 64, "test_size": 300, "device": "cpu"})
    hooks = ["mod.layer3.mod.0.mod.conv1.hook_point", "mod.layer1.mod.1.mod.conv2.hook_point"]
    res = {}
    for eng in ("native", "reference"):
        torch.manual_seed(0)
        res[eng] = evaluate_model_on_probes(ll, "pvr_leaky", {"batch_size": 32, "lr": 1e-3, "num_workers": 0,
                                                              "epochs": 1, "engine": eng},
                                            tr.base_data, te.base_data, hook_points=hooks)
    for h in hooks:
        a, b = res["native"][h]["test accuracy"], res["reference"][h]["test accuracy"]
        assert set(a) == set(b) and len(a) == 12
        assert max(abs(a[k] - b[k]) for k in a) <= 1e-6, (h, a, b)
        la, lb = res["native"][h]["test loss"], res["reference"][h]["test loss"]
        assert max(abs(la[k] - lb[k]) for k in la) <= 1e-4 * max(1.0, max(abs(v) for v in lb.values())), (h, la, lb)


def test_probe_bank_over_budget_falls_back(monkeypatch, capsys):
    """an activation bank above the memory budget is not built; the per-batch path gives the same result."""
    from iit_amd.entry.eval_information import evaluate_model_on_probes
    from iit_amd.tasks.task_loader import get_dataset
    from iit_amd.utils.probes import ActivationBank
    ll, _ = _setup(8)
    tr, te = get_dataset("pvr_leaky", dataset_config={"train_size": 32, "test_size": 64, "device": "cpu"})
    hooks = ["mod.layer3.mod.0.mod.conv1.hook_point"]
    need = ActivationBank.estimate_bytes(ll, tr.base_data, hooks)
    assert need > 32 * 100  # a layer-3 activation per sample, 32 samples
    res = {}
    for budget in ("100", "1e-6"):
        monkeypatch.setenv("IIT_PROBE_BANK_GB", budget)
        torch.manual_seed(0)
        res[budget] = evaluate_model_on_probes(ll, "pvr_leaky", {"batch_size": 16, "lr": 1e-3, "num_workers": 0,
                                                                 "epochs": 1, "engine": "native"},
                                               tr.base_data, te.base_data, hook_points=hooks)
    assert "per-batch capture instead" in capsys.readouterr().out
    a, b = res["100"][hooks[0]]["test accuracy"], res["1e-6"][hooks[0]]["test accuracy"]
    assert max(abs(a[k] - b[k]) for k in a) <= 1e-6
