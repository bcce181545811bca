"""Patch-spec splice (csrc/splice.hip, iit_amd.ops.splice): the reference's ``out = act.clone(); out[idx] = src[idx]``
hook (/root/reference/iit/model_pairs/base_model_pair.py:151-163) and StopGrad's scale / zero-grad hooks
(/root/reference/iit/model_pairs/stop_grad_pair.py:37-75) as one range-table kernel launch per site."""
import pytest
import torch

from iit_amd.core.index import Ix, TorchIndex

INDICES = [
    (Ix[:, -1, :2, :], (4, 16, 4, 32)),          # causal graph: last position, first head half
    (Ix[:, -1, 2:], (4, 16, 4, 32)),              # ... second half (trailing dim omitted)
    (Ix[:, [1, 2, 3, 7]], (8, 16, 64)),           # MQNLI: position list on [B, S, d]
    (Ix[:, -1, :96], (8, 16, 192)),               # MLP neurons at the last position
    (Ix[None, None, 0:3, 3:6], (2, 8, 6, 6)),     # PVR spatial quadrant (innermost dim 6: scalar path)
    (Ix[None, 16:32, None, None], (2, 64, 6, 6)),  # PVR channel quarter
    (Ix[:, :, 3], (4, 16, 8, 16)),                # one head
    (Ix[[None]], (4, 16, 32)),                    # everything
    (Ix[2:5], (8, 24)),                           # batch range, 2-D
    (Ix[:, :, [0, 2], :], (2, 4, 4, 8, 16)),      # 5-D hook: trailing whole dims collapse
]


def _mask_from_ranges(shape, ranges):
    m = torch.ones(shape, dtype=torch.bool)
    for d, runs in enumerate(ranges):
        sel = torch.zeros(shape[d], dtype=torch.bool)
        for lo, hi in runs:
            sel[lo:hi] = True
        view = [1] * len(shape)
        view[d] = shape[d]
        m &= sel.view(view)
    return m


@pytest.mark.parametrize("index,shape", INDICES)
def test_to_ranges_matches_torch_indexing(index, shape):
    ref = torch.zeros(shape, dtype=torch.bool)
    ref[index.as_index] = True
    ranges = index.to_ranges(shape)
    assert ranges is not None
    assert torch.equal(_mask_from_ranges(shape, ranges), ref)


def test_to_ranges_rejects_what_it_cannot_express():
    assert Ix[[0, 1], [1, 2]].to_ranges((4, 8)) is None  # paired list atoms (torch zips them)
    assert TorchIndex([slice(0, 8, 2)]).to_ranges((8,)) is None  # stepped slice
    assert Ix[:, :, :, :, 1].to_ranges((2, 2, 2, 2)) is None  # more atoms than dims
    assert Ix[:, list(range(0, 40, 2))].to_ranges((2, 64)) is None  # 20 runs > 8


def _ref_splice(act, index, src):
    out = act.clone()
    out[index.as_index] = src.expand_as(act)[index.as_index]
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("index,shape", INDICES)
def test_fused_splice_forward_backward(index, shape, dtype):
    """Forward equals clone + index_put exactly; the gradient is the incoming gradient with the spliced elements
    zeroed (the source is a detached constant), exactly as autograd differentiates the reference hook."""
    from iit_amd.ops import splice as sp
    torch.manual_seed(0)
    act = torch.randn(shape, device="cuda", dtype=dtype, requires_grad=True)
    src = torch.randn(shape, device="cuda", dtype=dtype)
    out = sp.splice(act, index, src)
    assert out is not None
    ref_act = act.detach().clone().requires_grad_(True)
    ref = _ref_splice(ref_act, index, src)
    assert torch.equal(out, ref)
    g = torch.randn(shape, device="cuda", dtype=dtype)
    out.backward(g)
    ref.backward(g)
    assert torch.equal(act.grad, ref_act.grad)
    sel = torch.zeros(shape, dtype=torch.bool, device="cuda")
    sel[index.as_index] = True
    assert not act.grad[sel].any()  # zero gradient through the spliced slice


@pytest.mark.gpu
def test_fused_splice_broadcast_source():
    """Mean-ablation style source: a [S, d] mean broadcast over the batch."""
    from iit_amd.ops import splice as sp
    act = torch.randn(8, 16, 64, device="cuda")
    src = torch.randn(16, 64, device="cuda")
    index = Ix[:, [0, 5, 6]]
    out = sp.splice(act, index, src)
    assert out is not None and torch.equal(out, _ref_splice(act, index, src))


@pytest.mark.gpu
def test_fused_divide_and_grad_mask():
    from iit_amd.core.index import EVERYTHING
    from iit_amd.ops import splice as sp
    x = torch.randn(4, 16, 8, 16, device="cuda", requires_grad=True)
    y = sp.divide(x, EVERYTHING, 1e6)
    assert torch.equal(y, x.detach() / 1e6)
    z = sp.grad_mask(y, [Ix[:, :, 3], Ix[:, :, 5]])
    z.backward(torch.ones_like(z))
    expect = torch.full_like(x, 1e-6)
    expect[:, :, 3] = 0
    expect[:, :, 5] = 0
    assert torch.equal(x.grad, expect)


def _splice_ops_during(fn):
    """aten ops of the reference's splice (``out[idx] = src[idx]``: a non-accumulating index_put) dispatched by ``fn``
    -- forward and backward; an embedding's gradient (an accumulating index_put) does not count."""
    from torch.utils._python_dispatch import TorchDispatchMode

    seen = []

    class Rec(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            kwargs = kwargs or {}
            name = str(func.overloadpacket)
            if name in ("aten.index_put", "aten.index_put_"):
                acc = args[3] if len(args) > 3 else kwargs.get("accumulate", False)
                if not acc:
                    seen.append(name)
            return func(*args, **kwargs)

    with Rec():
        fn()
    return seen


@pytest.mark.gpu
def test_causal_graph_step_has_no_index_put_splice():
    """The causal-graph correspondence splices token positions of hook_embed, last-position head halves of hook_z
    and MLP neurons (tasks/causal_graph make_causal_graph_corr): on the GPU every site runs the patch-spec kernel or
    (hook_z of the paired forward) the attention kernel's in-store splice, so a whole Strict-IIT step dispatches no
    splice index_put, while a fused kernel does launch."""
    from iit_amd.data.iit_dataset import IITDataset
    from iit_amd.models.transformer import HookedTransformer
    from iit_amd.ops import hip_kernels as K
    from iit_amd.tasks import causal_graph as cg

    cfg = dict(n_layers=4, d_model=128, n_heads=4, d_head=32, d_mlp=256, n_ctx=32, d_vocab=64, act_fn="gelu_new",
               normalization_type="LN", device="cuda", dtype=torch.bfloat16, positional_embedding_type="standard")
    torch.manual_seed(0)
    ll = HookedTransformer(cfg)
    ll.set_op_backend("hip")
    ds, hl, corr = cg.make_causal_graph_task(ll, n_samples=256, device="cuda")
    train = IITDataset(ds, ds, seed=0, device="cuda")
    pair = cg.CausalGraphModelPair(hl, ll, corr, training_args={"batch_size": 64, "lr": 1e-3, "lr_scheduler": None})
    opt = pair.make_optimizer(1e-3)
    base, abl = next(iter(train.make_loader(64, 0)))
    launches = []
    orig, orig_attn, orig_sparse = K.splice, K.attn_pair_fwd_spec, K.sparse_pair
    K.splice = lambda *a, **k: (launches.append(1), orig(*a, **k))[1]
    # hook_z sites of the paired forward splice inside the attention kernel's store, mlp.hook_post sites inside the
    # W_in op (sparse copy): fused launches too
    K.attn_pair_fwd_spec = lambda *a, **k: (launches.append(2), orig_attn(*a, **k))[1]
    K.sparse_pair = lambda *a, **k: (launches.append(3), orig_sparse(*a, **k))[1]
    try:
        for node in list(pair.corr.keys()):
            pair.sample_hl_name = lambda node=node: node
            pair.run_train_step(base, abl, pair.loss_fn, opt)  # warm-up: GEMM autotuning etc.
            launches.clear()
            bad = _splice_ops_during(lambda: pair.run_train_step(base, abl, pair.loss_fn, opt))
            assert not bad, (node, bad)
            assert launches, node  # the LL splice ran on a fused kernel
    finally:
        K.splice, K.attn_pair_fwd_spec, K.sparse_pair = orig, orig_attn, orig_sparse


@pytest.mark.gpu
def test_splice_channels_last_keeps_layout_and_matches_nchw():
    """SpliceFn on a channels-last activation splices in memory order (range table permuted to N, H, W, C): the
    output stays channels-last and equals the NCHW splice; the backward zeroes the same elements."""
    from iit_amd.core.index import Ix
    from iit_amd.ops import splice as sp
    torch.manual_seed(0)
    x = torch.randn(4, 64, 11, 11, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    src = torch.randn(4, 64, 11, 11, device="cuda").bfloat16()
    idx = Ix[None, 8:40, :5, 5:10]
    xa = x.detach().clone().requires_grad_()
    xb = x.detach().contiguous().requires_grad_()
    ya = sp.splice(xa, idx, src)
    yb = sp.splice(xb, idx, src)
    assert ya.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(ya, yb)
    g = torch.randn_like(yb)
    ya.backward(g)
    yb.backward(g)
    assert torch.equal(xa.grad, xb.grad)
    exp = g.clone()
    exp[idx.as_index] = 0
    assert torch.equal(xb.grad, exp)
