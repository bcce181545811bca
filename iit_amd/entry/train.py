"""MNIST-PVR training with IITBehaviorModelPair (parity: ``/root/reference/train.py:1-25``).

    python train.py                                   # 60k/10k, lr 1e-3, 10 epochs (reference config)
    python train.py --train-size 2048 --test-size 512 --epochs 1
"""
from __future__ import annotations

import argparse
import os

import torch

from iit_amd.model_pairs import IITBehaviorModelPair
from iit_amd.parallel import dist as pdist
from iit_amd.tasks.task_loader import get_alignment, get_dataset


def parse(argv=None):
    ap = argparse.ArgumentParser(description="IIT training on MNIST-PVR")
    ap.add_argument("--task", default="mnist_pvr", choices=["mnist_pvr", "pvr_leaky"])
    ap.add_argument("--train-size", type=int, default=60000)
    ap.add_argument("--test-size", type=int, default=10000)
    ap.add_argument("--batch-size", type=int, default=256)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--epochs", type=int, default=10)
    ap.add_argument("--mode", default="q", choices=["q", "c"])
    ap.add_argument("--hook-point", default="mod.layer3.mod.1.mod.conv2.hook_point")
    ap.add_argument("--wandb", action="store_true")
    ap.add_argument("--save", default=None, help="write the LL state_dict here (reference: weights/ll_model/{task}.pt)")
    ap.add_argument("--conv-benchmark", type=int, default=0,
                    help="1: MIOpen find mode (torch.backends.cudnn.benchmark) -- the fastest measured convolution "
                         "solution per shape (the bf16 PVR step 12.5 -> 9.0 ms, profiles/pvr_step_r5.txt), at a "
                         "first-call search cost of ~50 s per process; the fp32 NHWC step gains 16.6 -> 14.5 ms, and "
                         "the reference config reaches its early stop in 21.4 s without vs 72.0 s with it "
                         "(profiles/train_py_pvr_r5.txt), so it is off by default (long runs: pass 1)")
    ap.add_argument("--channels-last", type=int, default=1,
                    help="1: NHWC ResNet on the GPU -- MIOpen's NHWC convolutions and the fused NHWC BatchNorm / pool "
                         "kernels (fp32 PVR step 18.9 -> 14.6 ms, profiles/bn_fp32_r5.txt)")
    return ap.parse_args(argv)


def main(argv=None):
    args = parse(argv)
    pdist.init_distributed()
    if torch.cuda.is_available():
        torch.backends.cudnn.benchmark = bool(args.conv_benchmark)
    training_args = {"lr": args.lr, "early_stop": True, "batch_size": args.batch_size}
    dataset_config = {"train_size": args.train_size, "test_size": args.test_size, "batch_size": args.batch_size,
                      "num_workers": 0}
    train_set, test_set = get_dataset(args.task, dataset_config=dataset_config)
    ll_model, hl_model, corr = get_alignment(args.task, config={"input_shape": test_set.base_data.get_input_shape(),
                                                                "mode": args.mode, "hook_point": args.hook_point})
    if args.channels_last and torch.cuda.is_available():
        ll_model.to(memory_format=torch.channels_last)  # (state_dict layout-independent: checkpoints interchange)
    model_pair = IITBehaviorModelPair(ll_model=ll_model, hl_model=hl_model, corr=corr, training_args=training_args)
    model_pair.train(train_set, test_set, epochs=args.epochs, use_wandb=args.wandb)
    if pdist.is_main():
        print("done training")
        if args.save:
            os.makedirs(os.path.dirname(args.save) or ".", exist_ok=True)
            torch.save({k: v.detach().clone() for k, v in ll_model.state_dict().items()}, args.save)
    pdist.destroy()
    return model_pair


if __name__ == "__main__":
    main()
