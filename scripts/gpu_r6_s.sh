#!/bin/bash
# multi-rank launch path at HEAD rehearsed on one GPU (two gloo ranks share the card): self-launch weak + strong
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s
mkdir -p $O
IIT_REHEARSE_ONE_GPU=1 IIT_DIST_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --steps 5 --warmup 2 > $O/weak.log 2>&1 || { echo weak failed; tail -30 $O/weak.log; exit 5; }
grep -E '^\{' $O/weak.log | cut -c1-330
IIT_REHEARSE_ONE_GPU=1 IIT_DIST_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --steps 5 --warmup 2 --global-batch 256 > $O/strong.log 2>&1 || { echo strong failed; tail -30 $O/strong.log; exit 6; }
grep -E '^\{' $O/strong.log | cut -c1-330
grep -h "\[bench\]\|\[ddp\]\|wire" $O/weak.log | head -5
