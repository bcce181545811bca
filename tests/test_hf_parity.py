"""T1 per model family: the native hooked models vs Hugging Face ``transformers`` implementations
(random init, converted weights; nothing downloaded).  GPT-2 (unfolded LN) and Llama (RMSNorm, rotary,
SwiGLU, grouped-query attention)."""
import pytest
import torch

transformers = pytest.importorskip("transformers")

from iit_amd.models import convert  # noqa: E402
from iit_amd.models.transformer import HookedTransformer  # noqa: E402


def test_gpt2_matches_hf():
    torch.manual_seed(0)
    hcfg = transformers.GPT2Config(n_layer=2, n_embd=64, n_head=4, vocab_size=97, n_positions=32,
                                   attn_pdrop=0.0, resid_pdrop=0.0, embd_pdrop=0.0)
    hf = transformers.GPT2LMHeadModel(hcfg).eval()
    model = HookedTransformer(convert.gpt2_cfg_from_hf(hcfg, device="cpu"))
    convert.load_converted(model, convert.gpt2_state_dict_from_hf(hf))
    tok = torch.randint(0, 97, (3, 11))
    with torch.no_grad():
        ref = hf(tok).logits
        out = model(tok)
    assert torch.allclose(out, ref, atol=1e-4, rtol=1e-4), (out - ref).abs().max()


@pytest.mark.parametrize("n_kv", [2, 4])
def test_llama_matches_hf(n_kv):
    torch.manual_seed(0)
    hcfg = transformers.LlamaConfig(hidden_size=64, intermediate_size=96, num_hidden_layers=2, num_attention_heads=4,
                                    num_key_value_heads=n_kv, vocab_size=101, max_position_embeddings=64,
                                    rms_norm_eps=1e-5, tie_word_embeddings=False)
    hf = transformers.LlamaForCausalLM(hcfg).eval()
    model = HookedTransformer(convert.llama_cfg_from_hf(hcfg, device="cpu"))
    convert.load_converted(model, convert.llama_state_dict_from_hf(hf))
    tok = torch.randint(0, 101, (2, 13))
    with torch.no_grad():
        ref = hf(tok).logits
        out, cache = model.run_with_cache(tok)
    assert torch.allclose(out, ref, atol=1e-4, rtol=1e-4), (out - ref).abs().max()
    # TL hook surface of the Llama family
    for name in ("blocks.0.attn.hook_rot_q", "blocks.0.attn.hook_rot_k", "blocks.1.mlp.hook_pre_linear",
                 "blocks.1.mlp.hook_post", "blocks.0.ln1.hook_normalized", "blocks.1.attn.hook_z"):
        assert name in cache, name
    assert cache["blocks.0.attn.hook_k"].shape[2] == n_kv
    assert not hasattr(model, "pos_embed")
    names = [n for n, _ in model.named_parameters()]
    assert ("blocks.0.attn._W_K" in names) == (n_kv != 4)


def test_llama_presets_and_iit_intervention_on_llama():
    """A Llama-family LL model runs the plan-driven intervention engine (capture + per-head splice)."""
    from iit_amd.core.index import Ix
    from iit_amd.engine.plan import RunPlan
    cfg = convert.llama_config_dict("llama-3-8b")
    assert (cfg["n_layers"], cfg["d_model"], cfg["n_key_value_heads"], cfg["d_mlp"]) == (32, 4096, 8, 14336)
    torch.manual_seed(0)
    m = HookedTransformer(convert.llama_config_dict("llama-tiny", device="cpu"))
    src, base = torch.randint(0, 512, (4, 9)), torch.randint(0, 512, (4, 9))
    cap = m.run_capture(src, ["blocks.0.attn.hook_z"])
    out = m(base, plan=RunPlan.with_splices([("blocks.0.attn.hook_z", Ix[:, :, 1, :], cap["blocks.0.attn.hook_z"])],
                                            logits="last"))

    def hook(z, hook):
        z = z.clone()
        z[:, :, 1] = cap["blocks.0.attn.hook_z"][:, :, 1]
        return z
    ref = m.run_with_hooks(base, fwd_hooks=[("blocks.0.attn.hook_z", hook)])[:, -1]
    assert torch.allclose(out, ref, atol=1e-5)


@pytest.mark.parametrize("head", ["cls", "mlm"])
def test_bert_matches_hf(head):
    from iit_amd.models.bert import HookedEncoder, bert_config_dict, from_hf_bert
    torch.manual_seed(0)
    hcfg = transformers.BertConfig(hidden_size=64, num_hidden_layers=2, num_attention_heads=4, intermediate_size=128,
                                   vocab_size=120, max_position_embeddings=64, num_labels=3,
                                   hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    hf = (transformers.BertForSequenceClassification(hcfg) if head == "cls" else transformers.BertForMaskedLM(hcfg))
    hf = hf.eval()
    cfg = bert_config_dict("bert-tiny", d_vocab=120, device="cpu")
    model = HookedEncoder(cfg, n_classes=3 if head == "cls" else None)
    convert.load_converted(model, from_hf_bert(hf))
    tok = torch.randint(0, 120, (3, 10))
    tt = torch.cat([torch.zeros(3, 5, dtype=torch.long), torch.ones(3, 5, dtype=torch.long)], dim=1)
    am = torch.ones(3, 10, dtype=torch.long)
    am[1, 8:] = 0
    with torch.no_grad():
        ref = hf(input_ids=tok, token_type_ids=tt, attention_mask=am).logits
        out = model(tok, token_type_ids=tt, attention_mask=am)
    if head == "mlm":
        ref, out = ref[am.bool()], out[am.bool()]
    assert torch.allclose(out, ref, atol=1e-4, rtol=1e-4), (out - ref).abs().max()
