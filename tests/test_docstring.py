"""Docstring HL golden values (reference: iit/tasks/docstring/test_docstring.py:8-52)."""
import torch

from iit_amd.tasks.docstring import ArgMoverHead, Docstring_HL, InductionHead


def nonzero_values(a):
    return torch.cat((a.nonzero(), a[a != 0][:, None]), dim=-1)


def test_induction_head():
    prev_tok_out = torch.tensor([[2, 2, 2], [4, 5, 6]])
    tokens = torch.tensor([[1, 2, 3], [20, 4, 4]])
    result = InductionHead()(tokens, prev_tok_out)
    assert result.shape == (2, 3)
    assert result.equal(torch.tensor([[-1, 1, -1], [-1, 20, 20]]))


def test_arg_mover_head():
    tokens = torch.tensor([[0, 1, 2, 3], [4, 5, 6, 7]])
    def_patterns = torch.tensor([[10, 10, 2, 3], [9, 9, 9, 7]])
    induction_output = torch.tensor([[5, 0, 10, 1], [10, 9, 9, 9]])
    logits = ArgMoverHead(d_vocab=8, logit_increase=50)(tokens, def_patterns, induction_output)
    assert logits.shape == (2, 4, 8)
    assert nonzero_values(logits).equal(torch.tensor([[0, 2, 0, 50], [1, 2, 4, 50], [1, 3, 4, 50], [1, 3, 5, 50]]))


def test_docstring_abc():
    token_map = {"load": 1, "size": 2, "files": 3, ",": 4, "param": 5}
    text = "load , size , files 9 10 param load 11 param size 12 13 12 param"
    tokens = torch.tensor([[int(token_map.get(t, t)) for t in text.split()]])
    model = Docstring_HL()
    logits = model((tokens, None, None))
    assert nonzero_values(logits[0, -1]).equal(torch.tensor([[3, 50]]))
    # setup() was called: the HL can be used in a model pair (reference Q: it could not)
    assert set(model.hook_dict) == {"hook_pre", "hook_prev1", "hook_prev2", "hook_prev_doc", "hook_induction",
                                    "hook_arg_mover"}


def test_arg_mover_no_matches_is_zero():
    """The reference crashes (IndexError on an empty match set); here it yields zero logits."""
    tokens = torch.tensor([[1, 2, 3]])
    out = ArgMoverHead(d_vocab=5)(tokens, torch.tensor([[7, 7, 7]]), torch.tensor([[8, 8, 8]]))
    assert out.abs().sum() == 0
