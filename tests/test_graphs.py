"""HIP-graph captured train steps (iit_amd.engine.graphs) reproduce the eager schedule."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"


def _setup(seed=0, dtype=torch.bfloat16):
    from iit_amd.data.iit_dataset import IITDataset
    from iit_amd.model_pairs import IOI_ModelPair
    from iit_amd.models.config import gpt2_config_dict
    from iit_amd.models.transformer import HookedTransformer
    from iit_amd.tasks.ioi import ioi_cfg, make_ioi_corr, make_ioi_dataset_and_hl
    cfg = gpt2_config_dict()
    cfg.update(ioi_cfg)
    cfg.update(device=dev, dtype=dtype)
    torch.manual_seed(seed)
    ll = HookedTransformer(cfg)
    if dtype == torch.float32:
        ll.set_op_backend("torch")  # the fp32 (reference-precision) path train_ioi.py takes
    ds, hl = make_ioi_dataset_and_hl(512, ll, device=dev)
    train = IITDataset(ds, ds, seed=0, device=dev)
    pair = IOI_ModelPair(hl, ll, make_ioi_corr(6), training_args={"batch_size": 64, "lr": 1e-3, "strict_weight": 0.4,
                                                                   "lr_scheduler": None})
    opt = pair.make_optimizer(1e-3)
    return pair, opt, train


def _run(mode, n_batches=10, reps=3, dtype=torch.bfloat16):
    from iit_amd.engine.graphs import GraphedTrainStep
    pair, opt, train = _setup(dtype=dtype)
    torch.manual_seed(1)
    batches = [b for _, b in zip(range(n_batches), train.make_loader(64, 0))]
    step, g = pair.run_train_step, None
    import contextlib
    ctx = contextlib.nullcontext()
    if mode == "graphs":
        g = step = GraphedTrainStep(pair, opt, pair.loss_fn)
        ctx = g.stream_context()  # the whole loop on the runner's stream, as bench.py / BaseModelPair.train run it
    losses = []
    with ctx:
        for base, abl in batches * reps:
            out = step(base, abl, pair.loss_fn, opt)
            losses.append(torch.stack([out[k] for k in sorted(out)]))
    torch.cuda.synchronize()
    return torch.stack(losses).cpu(), g


# Graph replays run the eager kernel sequence, so losses agree phase by phase -- until fp32-atomic
# accumulation-order noise, which Adam amplifies (it normalises near-zero gradient elements to lr-sized
# steps), makes ANY two runs drift apart; on this config two eager runs split visibly after ~20 steps
# (scripts/diag_nondet.py).  So compare the first 12 steps (36 phases: every phase key captured and
# replayed at least once) tightly.
_TIGHT = 12


def test_graphed_steps_match_eager():
    le, _ = _run("eager")
    lg, g = _run("graphs")
    assert g.captures > 0 and g.replays > 0 and not g.failed, g.failed
    assert torch.allclose(le[:_TIGHT], lg[:_TIGHT], rtol=2e-3, atol=2e-3), (le[:_TIGHT] - lg[:_TIGHT]).abs().max()


def test_graphed_steps_match_eager_fp32_torch_backend():
    """The fp32 torch-op backend (train_ioi.py's reference-precision configuration) captured per phase, the loop
    on the runner's stream: every step reproduces the eager run bit for bit (no atomics on this path).  Regression
    for (a) autograd's AccumulateGrad running outside the capture when its node was made on another stream (the
    replays silently lost those gradient accumulations), (b) replays going stale when each step handed work
    between the caller's stream and the runner's (scripts/diag_graph_node.py)."""
    le, _ = _run("eager", dtype=torch.float32)
    lg, g = _run("graphs", dtype=torch.float32)
    assert g.captures > 0 and g.replays > 0 and not g.failed, g.failed
    err = (le - lg).abs().max(dim=1).values
    assert torch.equal(le, lg), [round(float(e), 6) for e in err]


def test_prime_captures_all_phase_keys_and_keeps_rng():
    from iit_amd.engine.graphs import GraphedTrainStep
    pair, opt, train = _setup()
    g = GraphedTrainStep(pair, opt, pair.loss_fn)
    base, abl = next(iter(train.make_loader(64, 0)))
    before = copy.deepcopy(pair.rng).random()
    n = g.prime(base, abl)
    assert n == len(pair.corr) + len(pair.nodes_not_in_circuit) + 1, g.failed
    assert pair.rng.random() == before


@pytest.mark.parametrize("staged", [False, True])
def test_split_graphs_for_data_parallel_match_eager(staged):
    """The DP form (graph[fwd+bwd] -> eager all-reduce -> graph[clip+Adam]) on one GPU (no-op reduce); with
    ``staged`` the backward is cut into per-stage graphs (engine/staged.py) exactly as data parallelism runs it."""
    from iit_amd.engine.graphs import GraphedTrainStep
    from iit_amd.engine.staged import staged_for
    le1, _ = _run("eager")
    pair, opt, train = _setup()
    torch.manual_seed(1)
    batches = [b for _, b in zip(range(10), train.make_loader(64, 0))]
    g = GraphedTrainStep(pair, opt, pair.loss_fn)
    g.split = True
    if staged:
        g.staged = staged_for(pair, 3)
        g.force_staged = True
        assert g.staged is not None and g.staged.cuts == [2, 4]
    losses = []
    for base, abl in batches * 3:
        out = g(base, abl, pair.loss_fn, opt)
        losses.append(torch.stack([out[k] for k in sorted(out)]))
    ls = torch.stack(losses).cpu()
    assert g.captures > 0 and not g.failed, g.failed
    if staged:
        assert all(len(ent[0][1]) == 2 for ent in g.graphs.values())  # two lower-stage graphs per phase
    assert torch.allclose(le1[:_TIGHT], ls[:_TIGHT], rtol=2e-3, atol=2e-3), (le1[:_TIGHT] - ls[:_TIGHT]).abs().max()



def _run_lr_change(mode, change_at=9, n_batches=6, reps=3):
    """fp32 torch-op backend (bit-exact graphs), the learning rate lowered 10x mid-run as ReduceLROnPlateau would."""
    from iit_amd.engine.graphs import GraphedTrainStep
    pair, opt, train = _setup(dtype=torch.float32)
    torch.manual_seed(1)
    batches = [b for _, b in zip(range(n_batches), train.make_loader(64, 0))]
    step, g = pair.run_train_step, None
    import contextlib
    ctx = contextlib.nullcontext()
    if mode == "graphs":
        g = step = GraphedTrainStep(pair, opt, pair.loss_fn)
        ctx = g.stream_context()
    losses = []
    with ctx:
        for i, (base, abl) in enumerate(batches * reps):
            if i == change_at:
                for grp in opt.param_groups:
                    grp["lr"] *= 0.1
            out = step(base, abl, pair.loss_fn, opt)
            losses.append(torch.stack([out[k] for k in sorted(out)]))
    torch.cuda.synchronize()
    return torch.stack(losses).cpu(), g


def test_graphed_steps_follow_lr_changes():
    """a captured Adam step must not keep the learning rate it saw at capture.  The fused kernel
    reads lr from a device scalar the runner refreshes before each replay, so a mid-run lr change (an LR scheduler
    between epochs) gives the eager trajectory bit for bit."""
    le, _ = _run_lr_change("eager")
    lg, g = _run_lr_change("graphs")
    assert g.captures > 0 and g.replays > 0 and not g.failed, g.failed
    assert torch.equal(le, lg), (le - lg).abs().max(dim=1).values
