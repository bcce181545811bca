"""Find nondeterminism: train eagerly, then re-evaluate one phase's forward several times (GPU)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch
from test_graphs import _setup

pair, opt, train = _setup()
torch.manual_seed(1)
batches = [b for _, b in zip(range(10), train.make_loader(64, 0))]
stop_at = int(os.environ.get("STOP", "64"))
count = [0]
target = {}
orig = pair.run_phase


def hooked(key, compute_loss, optimizer, step_fn):
    if count[0] == stop_at:
        target["key"] = key
        target["fn"] = compute_loss
        raise StopIteration
    count[0] += 1
    return orig(key, compute_loss, optimizer, step_fn)


pair.run_phase = hooked
try:
    for base, abl in batches * 3:
        pair.run_train_step(base, abl, pair.loss_fn, opt)
except StopIteration:
    pass
print("phase", stop_at, target["key"])
vals = []
with torch.no_grad():
    for i in range(6):
        vals.append(float(target["fn"]()))
print("repeat forward losses:", vals)
# per-op determinism of the pieces
from iit_amd.engine.plan import RunPlan
base, abl = batches[(stop_at // 3) % 10]
node = [n for n in pair.nodes_not_in_circuit if repr(n.index) == target["key"][2] and n.name == target["key"][1]]
if node:
    node = node[0]
    caps = [pair.ll_source_cache(abl[0], [node])[node.name].float().clone() for _ in range(3)]
    print("source capture max diff:", max((c - caps[0]).abs().max().item() for c in caps))
    outs = []
    for _ in range(3):
        pair.ll_cache = pair.ll_source_cache(abl[0], [node])
        outs.append(pair.ll_intervened_forward(base[0], [node]).float().clone())
    print("intervened logits max diff:", max((o - outs[0]).abs().max().item() for o in outs))
    plain = [pair.ll_model(base[0], plan=RunPlan(logits="last")).float().clone() for _ in range(3)]
    print("plain logits max diff:", max((o - plain[0]).abs().max().item() for o in plain))
