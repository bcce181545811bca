"""Fused gradient norm: the weight-gradient GEMMs add the sums of squares of the gradients they store, and the
optimizer's norm pass skips those slots (FlatParams.norm_cover / norm_spans)."""
import pytest
import torch


def _tiny_flat():
    from iit_amd.engine.flat import FlatParams

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = torch.nn.Parameter(torch.randn(8, 16))
            self.b = torch.nn.Parameter(torch.randn(16))
            self.c = torch.nn.Parameter(torch.randn(100, 8))

    m = M()
    return m, FlatParams(m)


def test_norm_spans_skip_covered_slots():
    """CPU: the norm spans are the arena minus the covered slots (with their padding); off -> plain pass."""
    m, flat = _tiny_flat()
    assert flat.norm_cover(m.a) is None  # fusion off by default
    flat.norm_fuse = True
    flat._norm_covered = {flat.index[id(m.a)]}
    flat.gsq = torch.zeros(64)
    tab, n, gsq = flat.norm_spans()
    assert gsq is flat.gsq and n > 0
    read = set()
    offs = dict((id(p), flat.offset_of(p)) for p in (m.a, m.b, m.c))
    for start4, local4, len4 in tab.view(-1, 3).tolist():
        assert start4 == local4
        read.update(range(start4 * 4, (start4 + len4) * 4))
    a0 = offs[id(m.a)]
    assert not read.intersection(range(a0, a0 + m.a.numel()))  # the covered slot is skipped
    for p in (m.b, m.c):
        assert set(range(offs[id(p)], offs[id(p)] + p.numel())) <= read  # the others are read
    assert flat._norm_covered == set()  # consumed
    assert flat.norm_spans() == (None, 0, None)  # nothing covered -> the plain pass


def test_norm_dirty_falls_back():
    m, flat = _tiny_flat()
    flat.norm_fuse = True
    flat.gsq = torch.ones(64)
    flat._norm_covered = {0}
    flat._norm_dirty = True
    assert flat.norm_spans() == (None, 0, None)
    assert float(flat.gsq.sum()) == 0.0  # stale sums dropped


@pytest.mark.gpu
def test_fused_norm_sums_match_gradients(monkeypatch):
    """GPU: in real IOI training steps, at every optimizer step the fused slots hold the sum of squares of exactly the
    covered weight gradients, and the rest of the norm pass skips them."""
    from iit_amd.data.iit_dataset import IITDataset
    from iit_amd.model_pairs import IOI_ModelPair
    from iit_amd.models.config import gpt2_config_dict
    from iit_amd.models.transformer import HookedTransformer
    from iit_amd.ops import hip_kernels
    from iit_amd.tasks.ioi import make_ioi_corr, make_ioi_dataset_and_hl

    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    cfg = gpt2_config_dict()
    cfg.update(n_layers=4, d_model=256, n_heads=4, d_head=64, d_mlp=1024, device="cuda:0", dtype=torch.bfloat16)
    ll = HookedTransformer(cfg)
    ll.set_op_backend("hip")
    ds, hl = make_ioi_dataset_and_hl(512, ll, device=dev)
    train = IITDataset(ds, ds, seed=0, device=dev)
    pair = IOI_ModelPair(hl, ll, make_ioi_corr(4),
                         training_args={"batch_size": 128, "lr": 1e-3, "lr_scheduler": None, "clip_grad_norm": 1.0})
    opt = pair.make_optimizer(1e-3)
    flat = opt.flat
    assert flat.norm_fuse  # single process: on by default
    checked = []
    real = hip_kernels.adam_step

    def checking_step(fl, *a, **kw):
        torch.cuda.synchronize()
        covered = set(fl._norm_covered)
        if covered and not fl._norm_dirty:
            want = 0.0
            for o, n in fl.slots:
                members = [i for i, p in enumerate(fl.params) if o <= fl.offset_of(p) < o + max(n, 1)]
                if members and all(i in covered for i in members):
                    want += float(fl.grad[o:o + n].double().pow(2).sum())
            got = float(fl.gsq.double().sum())
            checked.append((got, want))
        return real(fl, *a, **kw)

    monkeypatch.setattr(hip_kernels, "adam_step", checking_step)
    it = iter(train.make_loader(128, 0))
    for _ in range(2):
        base, abl = next(it)
        pair.run_train_step(base, abl, pair.loss_fn, opt)
    torch.cuda.synchronize()
    assert len(checked) >= 4, checked  # every optimizer phase of both steps took the fused path
    for got, want in checked:
        assert want > 0 and abs(got - want) <= 1e-4 * want, (got, want)
    assert float(flat.gsq.abs().sum()) == 0.0  # consumed and re-zeroed by the norm pass


@pytest.mark.gpu
def test_fused_norm_torch_backend_llama(monkeypatch):
    """GPU, torch op backend (Llama family): the weight-gradient GEMMs of ``_MirrorLinear`` / ``_MirrorMat``
    (``gemm_dispatch.wgrad_into(..., params=...)``) add the sums of squares of the gradients they store; at every
    optimizer step the slots hold exactly those, and the clip reads only the rest."""
    from iit_amd.data.iit_dataset import IITDataset
    from iit_amd.models.convert import llama_config_dict
    from iit_amd.models.transformer import HookedTransformer
    from iit_amd.ops import hip_kernels
    from iit_amd.tasks.causal_graph import CausalGraphModelPair, make_causal_graph_task

    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    cfg = llama_config_dict("llama-tiny", device="cuda:0", dtype=torch.bfloat16)
    ll = HookedTransformer(cfg)
    ds, hl, corr = make_causal_graph_task(ll, n_samples=256, device=dev, seq_len=24)
    pair = CausalGraphModelPair(hl, ll, corr, training_args={"batch_size": 32, "lr": 1e-4, "lr_scheduler": None,
                                                             "early_stop": False, "clip_grad_norm": 1.0})
    opt = pair.make_optimizer(1e-4)
    flat = opt.flat
    assert flat.norm_fuse
    checked = []
    real = hip_kernels.adam_step

    def checking_step(fl, *a, **kw):
        torch.cuda.synchronize()
        covered = set(fl._norm_covered)
        if covered and not fl._norm_dirty:
            want = 0.0
            for o, n in fl.slots:
                members = [i for i, p in enumerate(fl.params) if o <= fl.offset_of(p) < o + max(n, 1)]
                if members and all(i in covered for i in members):
                    want += float(fl.grad[o:o + n].double().pow(2).sum())
            checked.append((float(fl.gsq.double().sum()), want))
        return real(fl, *a, **kw)

    monkeypatch.setattr(hip_kernels, "adam_step", checking_step)
    train = IITDataset(ds, ds, seed=0, device=dev)
    it = iter(train.make_loader(32, 0))
    for _ in range(2):
        base, abl = next(it)
        pair.run_train_step(base, abl, pair.loss_fn, opt)
    torch.cuda.synchronize()
    assert len(checked) >= 4, checked
    for got, want in checked:
        assert want > 0 and abs(got - want) <= 1e-4 * want, (got, want)
