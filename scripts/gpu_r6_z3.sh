#!/bin/bash
# 6L/64d, seed 0, every 50 epochs: HIP bf16 engine vs the torch-op backend in bf16 (precision vs kernels), 300 epochs each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6z
mkdir -p $O
for be in hip torch-bf16; do
  timeout -k 10 560 python3 -u scripts/iia_ceiling.py --model ioi-6l --epochs 300 --every 50 --seed 0 --backend $be > $O/6l_s0_${be}_300.log 2>&1 || { tail -20 $O/6l_s0_${be}_300.log; exit 1; }
  grep -E '"metric"' $O/6l_s0_${be}_300.log | cut -c1-420
done
