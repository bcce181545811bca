#!/bin/bash
# 6L/64d, seed 0: is the bf16 failure to learn compute precision, or the fused-optimizer machinery the bf16 runs share
# (flat arena + bf16 mirror + clip norm fused into the weight-gradient GEMMs)?  torch-op backend in bf16, 160 epochs:
#   plain:  torch.optim.Adam on the module parameters (no arena, no mirror, no fused norm), eager phases
#   nonorm: fused Adam + mirror, but the clip norm from its own pass (IIT_FUSED_NORM=0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6z5
mkdir -p $O
timeout -k 10 560 python3 -u scripts/iia_ceiling.py --model ioi-6l --epochs 160 --every 40 --seed 0 --backend torch-bf16 \
  --plain-adam --graphs 0 > $O/plain.log 2>&1 || { tail -20 $O/plain.log; exit 1; }
grep -E '"metric"' $O/plain.log | cut -c1-600
IIT_FUSED_NORM=0 timeout -k 10 400 python3 -u scripts/iia_ceiling.py --model ioi-6l --epochs 160 --every 40 --seed 0 \
  --backend torch-bf16 > $O/nonorm.log 2>&1 || { tail -20 $O/nonorm.log; exit 1; }
grep -E '"metric"' $O/nonorm.log | cut -c1-600
