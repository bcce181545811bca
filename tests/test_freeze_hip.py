"""Frozen matrices on the HIP backend (``requires_grad=False`` W_O / W_in / W_out outside the flat arena): the bf16
mirror binds a copy of each frozen matrix, the forward matches the fp32 torch-op oracle, a training step leaves the
frozen matrices bitwise unchanged and moves the others, and an out-of-band edit of a frozen matrix reaches the
next forward.  Used by scripts/iia_ceiling.py ``--control zero-wo``."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _model(dtype):
    from iit_amd.models.transformer import HookedTransformer
    cfg = dict(n_layers=2, d_model=64, n_heads=4, d_head=16, d_mlp=256, n_ctx=16, d_vocab=97, act_fn="gelu",
               normalization_type="LN", device="cuda", init_weights=True, dtype=dtype, seed=0)
    return HookedTransformer(cfg)


def test_frozen_wo_and_mlp_on_hip_backend():
    from iit_amd.engine.flat import FlatParams
    torch.manual_seed(0)
    fast = _model(torch.bfloat16)
    ref = _model(torch.float32).set_op_backend("torch")
    ref.load_state_dict(fast.state_dict())
    frozen = [fast.blocks[0].attn.W_O, fast.blocks[1].mlp.W_in]
    with torch.no_grad():
        fast.blocks[0].attn.W_O.zero_()
        ref.blocks[0].attn.W_O.zero_()
    for p in frozen:
        p.requires_grad_(False)
    fast.mark_weights_changed()
    flat = FlatParams(fast, with_bf16_shadow=True)
    fast._flat_params = flat
    assert all(not flat.owns(p) for p in frozen)
    assert fast.ops().name == "hip"
    toks = torch.randint(0, 97, (8, 16), device="cuda")
    y = fast(toks).float()
    yr = ref(toks).float()
    assert float((y - yr).norm() / yr.norm()) < 2e-2
    before = [p.detach().clone() for p in frozen]
    others = {n: p.detach().clone() for n, p in fast.named_parameters() if p.requires_grad}
    opt = torch.optim.Adam([p for p in fast.parameters() if p.requires_grad], lr=1e-2)
    loss = fast(toks).float().logsumexp(-1).mean()
    loss.backward()
    flat.rebind_grads(zero_missing=True) if hasattr(flat, "rebind_grads") else None
    opt.step()
    fast.mark_weights_changed()
    for p, b in zip(frozen, before):
        assert torch.equal(p, b) and p.grad is None
    assert sum(int(not torch.equal(p, others[n])) for n, p in fast.named_parameters() if p.requires_grad) > 0
    with torch.no_grad():  # an out-of-band edit of a frozen matrix reaches the next forward
        fast.blocks[1].mlp.W_in.mul_(0.5)
        ref.load_state_dict(fast.state_dict())
    fast.mark_weights_changed()
    y = fast(toks).float()
    yr = ref(toks).float()
    assert float((y - yr).norm() / yr.norm()) < 2e-2
