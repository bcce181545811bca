"""The fused IOI HL label kernel (csrc/ioi_hl.hip) against the IOI_HL torch model under the reference's hook-based
interchange (/root/reference/iit/model_pairs/base_model_pair.py:120-150): the intervened label argmax(hl_out[:, -1])
for every HL node, on the synthetic IOI prompts and on adversarial random token sequences (repeats, names,
all-negative logits where the label is the smallest untouched vocabulary index)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _pair(n=512):
    from iit_amd.model_pairs import IOI_ModelPair
    from iit_amd.models.transformer import HookedTransformer
    from iit_amd.tasks.ioi import NAMES, make_ioi_corr, make_ioi_dataset_and_hl
    cfg = dict(n_layers=2, d_model=64, n_heads=4, d_head=16, d_mlp=128, n_ctx=16, d_vocab=50257, act_fn="gelu_new",
               normalization_type="LNPre", device="cuda", dtype=torch.bfloat16)
    ll = HookedTransformer(cfg)
    ds, hl = make_ioi_dataset_and_hl(n, ll, NAMES, device="cuda")
    return IOI_ModelPair(hl, ll, make_ioi_corr(2), training_args={"lr_scheduler": None}), ds


def _hook_label(pair, base, src, node):
    hl = pair.hl_model
    with torch.no_grad():
        _, pair.hl_cache = hl.run_with_cache((src,), last_only=True)
        out = hl.run_with_hooks((base,), fwd_hooks=[(node.name, pair.make_hl_ablation_hook(node))], last_only=True)
    return pair._hl_label(out)


def test_fast_label_matches_hooked_hl_on_ioi_prompts():
    pair, ds = _pair()
    x = ds.prompts[:, :-1].cuda()  # model inputs (the last token is the target)
    base, src = x[:256], x[256:512]
    for node in pair.corr.keys():
        fast = pair.fast_hl_label(base, src, node)
        assert fast is not None, node
        assert torch.equal(fast, _hook_label(pair, base, src, node)), node


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_fast_label_matches_hooked_hl_on_random_tokens(seed):
    pair, _ = _pair(64)
    names = pair.hl_model.name_mover_head.names.cuda()
    g = torch.Generator(device="cuda").manual_seed(seed)
    B, S = 512, 16
    # a mix of name tokens (repeated: duplicates / inhibition) and low vocabulary ids (collisions with index 0..)
    pick = torch.randint(0, names.numel(), (2, B, S), device="cuda", generator=g)
    low = torch.randint(0, 6, (2, B, S), device="cuda", generator=g)
    use_name = torch.rand(2, B, S, device="cuda", generator=g) < 0.6
    toks = torch.where(use_name, names[pick].long(), low)
    for node in pair.corr.keys():
        fast = pair.fast_hl_label(toks[0], toks[1], node)
        assert torch.equal(fast, _hook_label(pair, toks[0], toks[1], node)), node


def test_fast_label_declines_with_live_hl_hooks():
    pair, ds = _pair(64)
    x = torch.randint(0, 100, (8, 16), device="cuda")
    node = list(pair.corr.keys())[0]
    pair.hl_model.hook_duplicate.add_hook(lambda t, hook: t)
    try:
        assert pair.fast_hl_label(x, x, node) is None
    finally:
        pair.hl_model.reset_hooks()
