"""Causal-effect sweeps (iit_amd.utils.eval_ablations / eval_metrics): native plan engine vs reference hooks."""
import pytest
import torch

from iit_amd.core.index import EVERYTHING, Ix, TorchIndex
from iit_amd.data.iit_dataset import IITDataset, IITUniqueDataset
from iit_amd.tasks.ioi import make_ioi_corr, make_ioi_dataset_and_hl
from iit_amd.utils import eval_ablations as ea
from iit_amd.utils.eval_metrics import accuracy_affected, kl_div


def _pair(n_layers=6):
    from iit_amd.model_pairs import IOI_ModelPair
    from iit_amd.models.config import gpt2_config_dict
    from iit_amd.models.transformer import HookedTransformer
    cfg = gpt2_config_dict()
    cfg.update(n_layers=n_layers, d_model=32, n_heads=4, d_head=8, d_mlp=64, device="cpu")
    torch.manual_seed(0)
    ll = HookedTransformer(cfg)
    ds, hl = make_ioi_dataset_and_hl(96, ll, device="cpu")
    pair = IOI_ModelPair(hl, ll, make_ioi_corr(n_layers), training_args={"batch_size": 32, "lr_scheduler": None})
    return pair, ds


def test_kl_div_matches_definition():
    torch.manual_seed(0)
    a = torch.randn(5, 7, 11)
    b = torch.randn(5, 7, 11).softmax(-1)  # already a pmf: used as-is
    kl = kl_div(a, b, Ix[:, -1])
    pa = a[:, -1].softmax(-1)
    pb = b[:, -1]
    assert torch.allclose(kl, (pb * (pb.log() - pa.log())).sum(-1), atol=1e-6)
    unchanged = torch.tensor([True, False, False, True, False])
    r = accuracy_affected(a, b, unchanged, Ix[:, -1])
    flips = (a[:, -1].argmax(-1) != b[:, -1].argmax(-1)).float() * (~unchanged).float()
    assert torch.isclose(r, flips.sum() / 3)


def test_resample_ablation_native_equals_reference():
    pair, ds = _pair()
    iit_set = IITDataset(ds, ds, seed=0, device="cpu")
    res = {}
    for engine in ("native", "reference"):
        pair.training_args["engine"] = engine
        torch.manual_seed(0)
        res[engine] = {**ea.check_causal_effect(pair, iit_set, batch_size=32, node_type="n"),
                       **ea.check_causal_effect(pair, iit_set, batch_size=32, node_type="c")}
    assert res["native"].keys() == res["reference"].keys()
    assert len(res["native"]) == 8 + 7  # [OBS] 8 nodes not in the IOI circuit; 7 corr LL nodes
    for node in res["native"]:
        assert abs(res["native"][node] - res["reference"][node]) < 1e-4, node
    torch.manual_seed(0)
    pair.training_args["engine"] = "native"
    acc = ea.check_causal_effect(pair, iit_set, batch_size=32, node_type="c",
                                 categorical_metric=ea.Categorical_Metric.ACCURACY)
    assert all(0.0 <= v <= 1.0 for v in acc.values())


def test_mean_and_zero_ablation_native_equals_reference(tmp_path):
    pair, ds = _pair()
    uni = IITUniqueDataset(ds, ds, seed=0, device="cpu")
    out = {}
    for engine in ("native", "reference"):
        pair.training_args["engine"] = engine
        torch.manual_seed(0)
        mean_cache = ea.get_mean_cache(pair, uni, batch_size=32)
        torch.manual_seed(0)
        za_n, za_c = (ea.check_causal_effect_on_ablation(pair, uni, batch_size=32, node_type=t, mean_cache=mean_cache)
                      for t in ("n", "c"))
        torch.manual_seed(0)
        zero = ea.check_causal_effect_on_ablation(pair, uni, batch_size=32, node_type="c", mean_cache=None)
        out[engine] = (mean_cache, za_n, za_c, zero)
    mc_n, mc_r = out["native"][0], out["reference"][0]
    for k in ("blocks.0.attn.hook_z", "blocks.3.mlp.hook_post"):
        assert torch.allclose(mc_n[k], mc_r[k], atol=1e-5)
    for i in (1, 2, 3):
        for node, v in out["native"][i].items():
            assert abs(v - out["reference"][i][node]) < 1e-3, node
    df = ea.make_combined_dataframe_of_results(out["native"][1], out["native"][2], out["native"][1], out["native"][2],
                                               use_mean_cache=True)
    assert list(df.columns) == ["node", "status", "resample_ablate_effect", "mean_ablate_effect"]
    ea.save_result(df, str(tmp_path / "results"), pair)
    assert (tmp_path / "results" / "results.csv").exists()
    assert (tmp_path / "results" / "meta.log").read_text().startswith("{")


def test_batched_sweeps_equal_the_per_node_path():
    """the native sweeps share one source capture / HL output / base forward per batch across
    all nodes; the scores equal the per-node native path (``resample_ablate_node`` / ``ablate_node``) exactly."""
    pair, ds = _pair()
    pair.training_args["engine"] = "native"
    iit_set = IITDataset(ds, ds, seed=0, device="cpu")
    nodes = list(ea._nodes(pair, "n")) + list(ea._nodes(pair, "c"))
    torch.manual_seed(0)
    base_in, abl_in = next(iter(iit_set.make_loader(32, 0)))
    per_node = {n: 0 for n in nodes}
    for n in nodes:
        ea.resample_ablate_node(pair, base_in, abl_in, n, per_node)
    batched = {n: 0 for n in nodes}
    ea.resample_ablate_nodes(pair, base_in, abl_in, nodes, batched)
    for n in nodes:
        assert torch.equal(torch.as_tensor(per_node[n]), torch.as_tensor(batched[n])), n
    uni = IITUniqueDataset(ds, ds, seed=0, device="cpu")
    mean_cache = ea.get_mean_cache(pair, uni, batch_size=32)
    (b,) = [next(iter(uni.make_loader(32, 0)))]
    nodes = ea._nodes(pair, "a", with_suffixes=True)
    per_node = {n: 0 for n in nodes}
    for n in nodes:
        ea.ablate_node(pair, b, n, per_node, mean_cache=mean_cache, use_mean_cache=True)
    batched = {n: 0 for n in nodes}
    ea.ablate_nodes(pair, b, nodes, batched, {nm: mean_cache[nm] for nm in {n.name for n in nodes}})
    for n in nodes:
        assert torch.equal(torch.as_tensor(per_node[n]), torch.as_tensor(batched[n])), n


def test_prefix_shared_sweep_equals_full_forwards(monkeypatch):
    """Resuming each node's spliced forward from the cached base residual at its block (``_BasePrefix``) gives the
    scores of full forwards from the tokens."""
    pair, ds = _pair()
    iit_set = IITDataset(ds, ds, seed=0, device="cpu")
    uni = IITUniqueDataset(ds, ds, seed=0, device="cpu")
    res = {}
    for flag in (False, True):
        monkeypatch.setattr(ea, "_PREFIX", flag)
        torch.manual_seed(0)
        r = dict(ea.check_causal_effect(pair, iit_set, batch_size=32, node_type="n"))
        za_not, za_in = ea.get_causal_effects_for_all_nodes(pair, uni, batch_size=32, use_mean_cache=True)
        r.update({("za", k): v for k, v in {**za_not, **za_in}.items()})
        res[flag] = r
    assert res[False].keys() == res[True].keys()
    for k in res[False]:
        assert abs(res[False][k] - res[True][k]) < 1e-5, k


def test_node_batched_sweep_equals_per_node_forwards(monkeypatch):
    """Nodes of one block sharing one forward over stacked copies of the batch (``_RowGroupSplice``) give the scores
    of one spliced forward per node, for the resample and the mean-ablation sweeps."""
    pair, ds = _pair()
    iit_set = IITDataset(ds, ds, seed=0, device="cpu")
    uni = IITUniqueDataset(ds, ds, seed=0, device="cpu")
    calls = []
    orig = ea._BasePrefix.forward_rows

    def counting(self, base_x, layer, n, plan):
        calls.append(n)
        return orig(self, base_x, layer, n, plan)

    monkeypatch.setattr(ea._BasePrefix, "forward_rows", counting)
    res = {}
    for rows in (0, 1 << 20):
        monkeypatch.setattr(ea, "_GROUP_ROWS", rows)
        torch.manual_seed(0)
        r = dict(ea.check_causal_effect(pair, iit_set, batch_size=32, node_type="n"))
        za_not, za_in = ea.get_causal_effects_for_all_nodes(pair, uni, batch_size=32, use_mean_cache=True)
        r.update({("za", k): v for k, v in {**za_not, **za_in}.items()})
        res[rows] = r
        if rows == 0:
            assert not calls
    assert calls and max(calls) > 1
    assert res[0].keys() == res[1 << 20].keys()
    for k in res[0]:
        assert abs(res[0][k] - res[1 << 20][k]) < 1e-5, k


def test_row_group_splice_touches_only_its_rows():
    act = torch.randn(6, 3, 4, 2)
    src_a = torch.randn(2, 3, 4, 2)
    mean = torch.randn(1, 3, 4, 2)
    spl = ea._RowGroupSplice()
    spl.groups.append((0, 2, TorchIndex([slice(None), slice(None), 1]), src_a))
    spl.groups.append((4, 6, EVERYTHING, mean))
    out = spl.apply(act)
    ref = act.clone()
    ref[0:2, :, 1] = src_a[:, :, 1]
    ref[4:6] = mean.expand(2, 3, 4, 2)
    assert torch.equal(out, ref)
    assert not torch.equal(out, act)


def test_start_at_layer_resumes_the_forward():
    pair, _ = _pair()
    m = pair.ll_model
    tok = torch.randint(0, 1000, (4, 10))
    full = m(tok)
    resid3 = m.run_capture(tok, ["blocks.3.hook_resid_pre"])["blocks.3.hook_resid_pre"]
    assert torch.allclose(m(resid3, start_at_layer=3), full, atol=1e-5)


@pytest.mark.gpu
def test_kl_rows_kernel_matches_kl_div():
    """csrc/kernels.hip kl_rows (one pass over LL logits and the HL pmf) gives kl_div's per-row KL for logits and
    for rows that are already pmfs, including a padded row stride (the unembed's fp32 output)."""
    from iit_amd.utils.eval_metrics import kl_div_from_stats, target_stats
    torch.manual_seed(0)
    dev = "cuda"
    V = 50257
    hl = torch.randn(37, V, device=dev) * 4
    ll_pad = torch.randn(37, V + 7, device=dev) * 3
    ll = ll_pad[:, :V]  # row stride V + 7
    stats = target_stats(hl)
    got = kl_div_from_stats(ll, stats)
    want = kl_div(ll, hl, EVERYTHING)
    assert torch.allclose(got, want, rtol=1e-4, atol=1e-5)
    pm = torch.softmax(torch.randn(37, V, device=dev), -1)
    got = kl_div_from_stats(pm, stats)
    want = kl_div(pm, hl, EVERYTHING)
    assert torch.allclose(got, want, rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
def test_kl_rows_kernel_masked_logits():
    """A -inf (masked) logit -- including as a thread's first element, where the running max is still -inf --
    adds nothing to the logsumexp (exp(-inf - -inf) made the whole row NaN).  With the target pmf zero
    on the masked entries the KL equals the KL over the unmasked columns."""
    from iit_amd.utils.eval_metrics import kl_div_from_stats, target_stats
    torch.manual_seed(1)
    dev = "cuda"
    V = 4099
    a = torch.randn(9, V, device=dev) * 3
    hl = torch.randn(9, V, device=dev) * 4
    masked = torch.zeros(V, dtype=torch.bool, device=dev)
    masked[:300] = True  # every thread's first element of row 0's stream (threads 0..255) and more
    masked[1000:1013] = True
    a[:, masked] = -float("inf")
    hl[:, masked] = -float("inf")  # target pmf exactly 0 there
    stats = target_stats(hl)
    got = kl_div_from_stats(a, stats)
    keep = ~masked
    want = kl_div(a[:, keep], hl[:, keep], EVERYTHING)
    assert torch.isfinite(got).all()
    assert torch.allclose(got, want, rtol=1e-4, atol=1e-5)
