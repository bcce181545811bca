"""Train an IOI model pair and save it in the reference checkpoint layout.

Parity: ``/root/reference/train_ioi.py:1-82`` (same training_args, seeds, 12k
samples, 80/20 split, ``IOI_ModelPair``, up to 1000 epochs, checkpoint files).
Additions: CLI flags, bf16/HIP engine selection, data parallelism (launch with
``torchrun --nproc-per-node N --master-addr 127.0.0.1 train_ioi.py``),
per-epoch resume checkpoints (``--checkpoint-dir`` / ``--resume``).

    python train_ioi.py                       # reference config (6L/4H/64d LL), fp32
    python train_ioi.py --model gpt2-small --dtype bf16 --epochs 5
"""
from __future__ import annotations

import argparse
import os

import numpy as np
import torch

from iit_amd import model_pairs as mp
from iit_amd.data.iit_dataset import IITDataset, train_test_split
from iit_amd.models.config import gpt2_config_dict
from iit_amd.models.transformer import HookedTransformer
from iit_amd.parallel import dist as pdist
from iit_amd.tasks.ioi import NAMES, ioi_cfg, make_ioi_corr, make_ioi_corr_dict, make_ioi_dataset_and_hl
from iit_amd.utils import checkpoint as ck


def parse(argv=None):
    ap = argparse.ArgumentParser(description="IIT training on IOI")
    ap.add_argument("--num-samples", type=int, default=12000)
    ap.add_argument("--epochs", type=int, default=1000)
    ap.add_argument("--batch-size", type=int, default=256)
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--iit-weight", type=float, default=1.0)
    ap.add_argument("--behavior-weight", type=float, default=1.0)
    ap.add_argument("--strict-weight", type=float, default=0.4)
    ap.add_argument("--use-single-loss", action="store_true")
    ap.add_argument("--no-early-stop", action="store_true")
    ap.add_argument("--model", default="ioi-6l", choices=["ioi-6l", "gpt2-small"])
    ap.add_argument("--dtype", default=None, choices=["fp32", "bf16"],
                    help="compute dtype (default: bf16 on GPU for gpt2-small, fp32 otherwise)")
    ap.add_argument("--engine", default="native", choices=["native", "reference"])
    ap.add_argument("--wandb", action="store_true")
    ap.add_argument("--save-root", default="models/ioi")
    ap.add_argument("--checkpoint-dir", default=None)
    ap.add_argument("--resume", action="store_true")
    ap.add_argument("--max-steps", type=int, default=None, help="cap on steps per epoch (smoke runs)")
    return ap.parse_args(argv)


def main(argv=None):
    args = parse(argv)
    pdist.init_distributed()
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    training_args = {
        "batch_size": args.batch_size,
        "lr": args.lr,
        "iit_weight": args.iit_weight,
        "behavior_weight": args.behavior_weight,
        "strict_weight": args.strict_weight,
        "next_token": False,
        "lr_scheduler": None,
        "clip_grad_norm": 1.0,
        "early_stop": not args.no_early_stop,
        "use_single_loss": args.use_single_loss,
        "engine": args.engine,
    }
    torch.manual_seed(0)
    np.random.seed(0)
    ll_cfg = gpt2_config_dict()
    if args.model == "ioi-6l":
        ll_cfg.update(ioi_cfg)
    dtype = args.dtype or ("bf16" if (dev.type == "cuda" and args.model == "gpt2-small") else "fp32")
    ll_cfg.update(init_weights=True, device=str(dev), dtype=torch.bfloat16 if dtype == "bf16" else torch.float32)
    ll_model = HookedTransformer(ll_cfg)
    if dtype == "fp32" or args.engine == "reference":
        ll_model.set_op_backend("torch")
    if pdist.is_main():
        print("making ioi dataset and hl")
    ioi_dataset, hl_model = make_ioi_dataset_and_hl(args.num_samples, ll_model, NAMES, verbose=False, device=dev)
    train_ds, test_ds = train_test_split(ioi_dataset, test_size=0.2, random_state=42)
    train_set = IITDataset(train_ds, train_ds, seed=0, device=dev)
    test_set = IITDataset(test_ds, test_ds, seed=0, device=dev)
    n_layers = ll_cfg["n_layers"]
    corr_dict = make_ioi_corr_dict(n_layers)
    model_pair = mp.IOI_ModelPair(ll_model=ll_model, hl_model=hl_model, corr=make_ioi_corr(n_layers),
                                  training_args=training_args)
    model_pair.train(train_set, test_set, epochs=args.epochs, use_wandb=args.wandb,
                     checkpoint_dir=args.checkpoint_dir, resume=args.resume, max_steps=args.max_steps)
    if pdist.is_main():
        print("done training")
        save_dir = ck.model_dir(model_pair, root=args.save_root)
        ck.save_reference_layout(save_dir, model_pair, epochs=args.epochs, corr_dict=corr_dict)
        print(f"saved to {save_dir}")
    pdist.destroy()


if __name__ == "__main__":
    main()
