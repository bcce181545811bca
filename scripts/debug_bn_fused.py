"""Why the fused BN path does or does not engage in the PVR family step (diagnostic)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from iit_amd.models import resnet as R
    from iit_amd.ops import bn as fbn
    from iit_amd.tasks.task_loader import get_alignment, get_dataset
    dev = torch.device("cuda")
    tr_set, te_set = get_dataset("mnist_pvr", {"train_size": 512, "test_size": 256, "device": dev})
    ll, hl, corr = get_alignment("mnist_pvr", {"input_shape": te_set.base_data.get_input_shape(), "device": dev})
    ll.to(memory_format=torch.channels_last)
    seen = []
    orig = R.fused_bn_act

    def probe(bn_m, relu_m, x, res=None):
        out = orig(bn_m, relu_m, x, res)
        if len(seen) < 6:
            bn = getattr(bn_m, "mod", bn_m)
            seen.append(dict(fused=out is not None, dtype=str(x.dtype), cl=x.is_contiguous(memory_format=torch.channels_last),
                             hooked=R._hooked(bn_m), relu_hooked=relu_m is not None and R._hooked(relu_m),
                             enabled=fbn.enabled(), covered=fbn.covered(x, bn, res) if x.is_cuda else None,
                             shape=tuple(x.shape), stride=tuple(x.stride())))
        return out
    R.fused_bn_act = probe
    x = tr_set.base_data.gather(torch.arange(0, 64, device=dev))[0].contiguous(memory_format=torch.channels_last)
    with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
        y = ll(x)
    print("plain forward:", seen[:2])
    seen.clear()
    from iit_amd.model_pairs import IITBehaviorModelPair
    pair = IITBehaviorModelPair(hl, ll, corr, training_args={"batch_size": 64, "lr": 1e-3, "lr_scheduler": None,
                                                              "early_stop": False})
    opt = pair.make_optimizer(1e-3)
    base, abl = next(iter(tr_set.make_loader(64, 0)))
    with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
        pair.run_train_step(base, abl, pair.loss_fn, opt)
    print("train step:")
    for s in seen:
        print(s)


if __name__ == "__main__":
    main()
