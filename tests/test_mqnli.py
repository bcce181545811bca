"""MQNLI natural-logic causal model + BERT encoder IIT (BASELINE.json config 4)."""
import torch

from iit_amd.data.iit_dataset import IITDataset, train_test_split
from iit_amd.models.bert import HookedEncoder, bert_config_dict
from iit_amd.tasks.mqnli import (CLS, EMPTY, H_POS, NOT, NODES, P_POS, Q0, SEP, MQNLI_HL, MQNLIDataset,
                                 make_mqnli_task)
from iit_amd.tasks.mqnli import natural_logic as nl


def _sent(q, adj, noun, neg, adv, verb):
    return [q, adj, noun, neg, adv, verb]


def _pair_tokens(p, h):
    return torch.tensor([[CLS] + p + [SEP] + h + [SEP]])


def test_natural_logic_golden_inferences():
    hl = MQNLI_HL()
    some, every, no, notevery = (Q0 + i for i in range(4))
    tall, dog, run, fast = 9, 17, 29, 25
    lab = lambda p, h: int(hl((_pair_tokens(p, h), None, None)).argmax(-1))  # noqa: E731
    # every tall dog runs  |=  some tall dog runs                            (entailment)
    assert lab(_sent(every, tall, dog, EMPTY, EMPTY, run), _sent(some, tall, dog, EMPTY, EMPTY, run)) == 0
    # some tall dog runs   |=  some dog runs                                  (upward restrictor)
    assert lab(_sent(some, tall, dog, EMPTY, EMPTY, run), _sent(some, EMPTY, dog, EMPTY, EMPTY, run)) == 0
    # every dog runs       |=  every tall dog runs                            (downward restrictor)
    assert lab(_sent(every, EMPTY, dog, EMPTY, EMPTY, run), _sent(every, tall, dog, EMPTY, EMPTY, run)) == 0
    # no dog runs fast  vs  some dog runs fast                                (contradiction)
    assert lab(_sent(no, EMPTY, dog, EMPTY, fast, run), _sent(some, EMPTY, dog, EMPTY, fast, run)) == 1
    # every dog runs  vs  every dog does not run                              (contradiction, non-empty restrictor)
    assert lab(_sent(every, EMPTY, dog, EMPTY, EMPTY, run), _sent(every, EMPTY, dog, NOT, EMPTY, run)) == 1
    # some dog runs  vs  some dog runs fast                                   (neutral)
    assert lab(_sent(some, EMPTY, dog, EMPTY, EMPTY, run), _sent(some, EMPTY, dog, EMPTY, fast, run)) == 2
    assert nl.quantifier_table()[nl.NO, nl.SOME, nl.EQ, nl.EQ] == nl.NEG


def test_dataset_balanced_and_consistent():
    ds = MQNLIDataset(900, seed=1, device="cpu")
    counts = torch.bincount(ds.y, minlength=3)
    assert counts.min() >= 250
    out, cache = MQNLI_HL().run_with_cache((ds.x, ds.y, ds.iv))
    assert torch.equal(out.argmax(-1), ds.y)
    for i, n in enumerate(NODES):
        assert torch.equal(cache[n], ds.iv[:, i]), n
    assert ds.x.shape[1] == 15 and (ds.x[:, 7] == SEP).all()


def test_bert_iit_on_mqnli_native_equals_reference_and_trains():
    from iit_amd.model_pairs import IITBehaviorModelPair
    torch.manual_seed(0)
    ll = HookedEncoder(bert_config_dict("bert-tiny", d_vocab=40, n_layers=4, device="cpu"), n_classes=3)
    ds, hl, corr = make_mqnli_task(ll, n_samples=384, device="cpu")
    pair = IITBehaviorModelPair(hl, ll, corr, training_args={"batch_size": 64, "lr": 1e-3, "lr_scheduler": None,
                                                              "early_stop": False})
    train = IITDataset(ds, ds, seed=0, device="cpu")
    base, abl = next(iter(train.make_loader(32, 0)))
    for hl_node in corr.keys():
        pair.training_args["engine"] = "native"
        l1 = pair.get_IIT_loss_over_batch(base, abl, hl_node, pair.loss_fn)
        pair.training_args["engine"] = "reference"
        l2 = pair.get_IIT_loss_over_batch(base, abl, hl_node, pair.loss_fn)
        assert torch.allclose(l1, l2, atol=1e-5), hl_node
    pair.training_args["engine"] = "native"
    tr, te = train_test_split(ds, 0.25, 42)
    pair.train(IITDataset(tr, tr, seed=0, device="cpu"), IITDataset(te, te, seed=0, device="cpu"), epochs=2)
    assert set(pair.test_metrics.to_dict()) >= {"val/IIA", "val/accuracy"}
