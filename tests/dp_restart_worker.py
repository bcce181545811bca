"""Worker of the multi-rank failure / restart rehearsal (tests/test_distributed.py::test_dp2_rank_failure_restart_resumes;
SURVEY.md §5.3: ``torchrun --max-restarts`` + resume + a hook that kills rank k at step n).

Run by ``python -m torch.distributed.run --nproc-per-node 2 --max-restarts 1 ... dp_restart_worker.py OUT FAULT``:
gloo data parallelism over 2 ranks trains the reference ``BaseModelPair.train`` loop for 3 epochs with a resume
checkpoint per epoch.  With FAULT = 1, rank 1 dies (``os._exit``, no clean-up, no exception) right after the epoch-0
checkpoint of the first attempt; torchrun tears the job down and restarts every rank, which resume from the
per-rank checkpoint (``TORCHELASTIC_RESTART_COUNT`` > 0).  Rank 0 writes the final weights and the attempt count.
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out_dir, fault = sys.argv[1], int(sys.argv[2])
    zero = len(sys.argv) > 3 and sys.argv[3] == "zero"
    from iit_amd.data.iit_dataset import IITDataset, train_test_split
    from iit_amd.model_pairs import IOI_ModelPair
    from iit_amd.models.config import gpt2_config_dict
    from iit_amd.models.transformer import HookedTransformer
    from iit_amd.parallel import dist as pdist
    from iit_amd.tasks.ioi import make_ioi_corr, make_ioi_dataset_and_hl
    from iit_amd.utils import checkpoint as ck
    pdist.init_distributed("gloo")
    torch.set_num_threads(1)
    rank = pdist.rank()
    attempt = int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"))
    cfg = gpt2_config_dict()
    cfg.update(n_layers=2, d_model=16, n_heads=2, d_head=8, d_mlp=32, device="cpu")
    torch.manual_seed(0)
    ll = HookedTransformer(cfg)
    ds, hl = make_ioi_dataset_and_hl(256, ll, device="cpu")
    args = {"batch_size": 32, "lr": 1e-3, "lr_scheduler": None, "early_stop": False, "strict_weight": 0.4,
            "bucket_mb": 0.05}
    if zero:
        args.update(zero=True, fused_optimizer=True)
    pair = IOI_ModelPair(hl, ll, make_ioi_corr(2), training_args=args)
    tr, te = train_test_split(ds, 0.25, 42)
    train, test = IITDataset(tr, tr, seed=0, device="cpu"), IITDataset(te, te, seed=0, device="cpu")
    ckdir = os.path.join(out_dir, "ck")

    def hook(epoch):
        if fault and attempt == 0 and rank == 1 and epoch == 0:
            sys.stdout.flush()
            os._exit(17)  # a hard rank failure: no exception, no collective clean-up

    pair.train(train, test, epochs=3, checkpoint_dir=ckdir, resume=ck.has_resume_state(ckdir), fault_hook=hook)
    if rank == 0:
        torch.save({"params": {n: p.detach().clone() for n, p in pair.ll_model.named_parameters()},
                    "attempt": attempt}, os.path.join(out_dir, "final.pt"))
    pdist.barrier()
    pdist.destroy()


if __name__ == "__main__":
    main()
