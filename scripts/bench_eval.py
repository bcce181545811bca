"""Evaluation throughput (IOI_ModelPair eval epoch: interchange intervention + IIA + per-token accuracy) on the
headline GPT-2-small config, with and without double-buffered source caches (iit_amd.engine.prefetch)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(batch=512, samples=12000, model="gpt2-small"):
    from iit_amd.data.iit_dataset import IITDataset
    from iit_amd.model_pairs import IOI_ModelPair
    from iit_amd.models.config import gpt2_config_dict
    from iit_amd.models.transformer import HookedTransformer
    from iit_amd.tasks.ioi import make_ioi_corr, make_ioi_dataset_and_hl
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    cfg = gpt2_config_dict()
    if model == "ioi-6l":  # the reference's own IOI LL model (6L / 64d / 4H)
        from iit_amd.tasks.ioi import ioi_cfg
        cfg.update(ioi_cfg)
    cfg.update(device="cuda:0", dtype=torch.bfloat16)
    ll = HookedTransformer(cfg)
    ds, hl = make_ioi_dataset_and_hl(samples, ll, device=dev)
    test = IITDataset(ds, ds, seed=0, device=dev)
    pair = IOI_ModelPair(hl, ll, make_ioi_corr(cfg["n_layers"]), training_args={"batch_size": batch, "lr_scheduler": None})
    res = {}
    for name, on in (("serial", False), ("prefetch", True), ("serial", False), ("prefetch", True)):
        pair.training_args["prefetch_source"] = on
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m = pair._run_eval_epoch(test.make_loader(batch, 0, shuffle=False), pair.loss_fn).to_dict()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res[name] = (len(test) / dt, float(m["val/IIA"]))
        print(f"{name:9s} {len(test) / dt:10.0f} pairs/s  ({dt * 1e3:7.1f} ms / {len(test)} pairs)  IIA {m['val/IIA']:.3f}",
              flush=True)
    print(f"{model}: speedup {res['prefetch'][0] / res['serial'][0]:.3f}x")


if __name__ == "__main__":
    main(model=sys.argv[1] if len(sys.argv) > 1 else "gpt2-small")
