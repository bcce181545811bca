"""The headline step's fused clip+Adam (restricted arena: the embedding rows no IOI token reaches are skipped) timed
alone, graph-replayed back to back, vs its in-step time from the kernel trace: bytes/s on the live parameters."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from iit_amd.data.iit_dataset import IITDataset, train_test_split
    from iit_amd.model_pairs import IOI_ModelPair
    from iit_amd.models.config import gpt2_config_dict
    from iit_amd.models.transformer import HookedTransformer
    from iit_amd.tasks.ioi import make_ioi_corr, make_ioi_dataset_and_hl
    dev = torch.device("cuda")
    torch.manual_seed(0)
    cfg = gpt2_config_dict()
    cfg.update(device=str(dev), init_weights=True, dtype=torch.bfloat16)
    ll = HookedTransformer(cfg)
    ds, hl = make_ioi_dataset_and_hl(12000, ll, device=dev)
    tr, _ = train_test_split(ds, test_size=0.2, random_state=42)
    train_set = IITDataset(tr, tr, seed=0, device=dev)
    pair = IOI_ModelPair(ll_model=ll, hl_model=hl, corr=make_ioi_corr(12),
                         training_args={"batch_size": 256, "lr": 1e-4, "clip_grad_norm": 1.0})
    opt = pair.make_optimizer(1e-4)
    pair.restrict_sparse_rows(train_set)
    flat = ll._flat_params
    base, abl = next(iter(train_set.make_loader(256, 0)))
    pair.run_train_step(base, abl, pair.loss_fn, opt)
    tab, n = flat.span_table()
    live = int(tab.view(-1, 3)[:, 2].sum().item()) * 4
    print(f"arena {flat.numel} params, live {live} in {n} spans", flush=True)
    flat.grad.normal_(std=1e-3)
    opt.step(clip_norm=1.0)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(10):
            opt.step(clip_norm=1.0)
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        s.record()
        g.replay()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / 10)
    print(f"isolated: {best * 1e3:.1f} us per clip+Adam step, {live * 30 / (best * 1e-3) / 1e12:.2f} TB/s at 30 B/param",
          flush=True)
    # the same pass after a 1 GiB sweep (cold L2 / Infinity Cache / TLB, as after the step's backward)
    junk = torch.empty(1 << 28, dtype=torch.float32, device=dev)
    times = []
    for _ in range(5):
        junk.add_(1.0)
        s.record()
        opt.step(clip_norm=1.0)
        e.record()
        e.synchronize()
        times.append(s.elapsed_time(e))
    print(f"after a 1 GiB sweep: {min(times) * 1e3:.1f} us", flush=True)


if __name__ == "__main__":
    main()
