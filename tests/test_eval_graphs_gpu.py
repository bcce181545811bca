"""Graph-captured evaluation sweeps and primed training graphs on the GPU, against their eager forms.

* ``IIT_EVAL_GRAPHS=1`` (``utils/eval_ablations._SweepGraph``): each sweep's per-batch body -- one source capture,
  one HL forward, one spliced forward + score per node -- captured once and replayed; the scores must equal the
  eager sweep's (``/root/reference/iit/utils/eval_ablations.py:128-161, 196-234`` semantics);
* ``prime_graphs`` (``BaseModelPair._prime_train_graphs``): every (phase, node) graph captured before epoch 0 with the
  training state restored, so training is the un-primed run's (``/root/reference/iit/model_pairs/
  base_model_pair.py:204-261``).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = torch.device("cuda")


def _pair(n_layers=4, samples=512):
    from iit_amd.model_pairs import IOI_ModelPair
    from iit_amd.models.config import gpt2_config_dict
    from iit_amd.models.transformer import HookedTransformer
    from iit_amd.tasks.ioi import make_ioi_corr, make_ioi_dataset_and_hl
    cfg = gpt2_config_dict()
    cfg.update(n_layers=n_layers, d_model=128, n_heads=4, d_head=32, d_mlp=512, device=str(dev), dtype=torch.bfloat16)
    torch.manual_seed(0)
    ll = HookedTransformer(cfg)
    ds, hl = make_ioi_dataset_and_hl(samples, ll, device=dev)
    pair = IOI_ModelPair(hl, ll, make_ioi_corr(n_layers), training_args={"batch_size": 64, "lr": 1e-3,
                                                                         "lr_scheduler": None, "early_stop": False})
    return pair, ds


def test_graphed_sweeps_equal_eager(monkeypatch):
    from iit_amd.data.iit_dataset import IITDataset, IITUniqueDataset
    from iit_amd.utils import eval_ablations as ea
    pair, ds = _pair()
    iit_set = IITDataset(ds, ds, seed=0, device=dev)
    uni = IITUniqueDataset(ds, ds, seed=0, device=dev)
    res = {}
    for g in ("0", "1"):
        monkeypatch.setenv("IIT_EVAL_GRAPHS", g)
        torch.manual_seed(0)
        r = {("n",) + (k.name, str(k.index)): v for k, v in
             ea.check_causal_effect(pair, iit_set, batch_size=64, node_type="n").items()}
        r.update({("c",) + (k.name, str(k.index)): v for k, v in
                  ea.check_causal_effect(pair, iit_set, batch_size=64, node_type="c").items()})
        za_not, za_in = ea.get_causal_effects_for_all_nodes(pair, uni, batch_size=64, use_mean_cache=True)
        r.update({("za",) + (k.name, str(k.index)): v for k, v in {**za_not, **za_in}.items()})
        res[g] = r
    assert res["0"].keys() == res["1"].keys() and len(res["0"]) > 0
    for k in res["0"]:
        assert abs(res["0"][k] - res["1"][k]) <= 1e-5 + 1e-3 * abs(res["0"][k]), (k, res["0"][k], res["1"][k])


def test_prime_preserving_restores_the_training_state():
    """Priming captures every (phase, node) graph and then puts weights, bf16 mirror, Adam moments, step counters and
    RNGs back bit for bit, so the run that follows is the unprimed run."""
    from iit_amd.data.iit_dataset import IITDataset
    from iit_amd.engine.graphs import GraphedTrainStep
    pair, ds = _pair(samples=512)
    train = IITDataset(ds, ds, seed=0, device=dev)
    opt = pair.make_optimizer(1e-3)
    loader = train.make_loader(64, 0)
    base, abl = next(iter(loader))
    pair.run_train_step(base, abl, pair.loss_fn, opt)  # non-zero moments and step counters
    flat = pair.ll_model._flat_params
    snap = {"data": flat.data.clone(), "shadow": flat.shadow.clone(), "m": opt.exp_avg.clone(),
            "v": opt.exp_avg_sq.clone(), "step": opt._step_dev.clone(), "cpu": torch.get_rng_state(),
            "cuda": torch.cuda.get_rng_state(), "count": opt.step_count}
    rng = pair.rng.bit_generator.state
    step = GraphedTrainStep(pair, opt, pair.loss_fn)
    with step.stream_context():
        n = step.prime_preserving(base, abl, pair.loss_fn, opt)
    torch.cuda.synchronize()
    assert n > 0 and step.captures > 0
    assert torch.equal(flat.data, snap["data"]) and torch.equal(flat.shadow, snap["shadow"])
    assert torch.equal(opt.exp_avg, snap["m"]) and torch.equal(opt.exp_avg_sq, snap["v"])
    assert torch.equal(opt._step_dev, snap["step"]) and opt.step_count == snap["count"]
    assert torch.equal(torch.get_rng_state(), snap["cpu"]) and torch.equal(torch.cuda.get_rng_state(), snap["cuda"])
    assert pair.rng.bit_generator.state == rng
