#!/bin/bash
# 6L/64d plateau exit, long runs: HIP bf16 engine 1000 epochs, seeds 0 and 1
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6z
mkdir -p $O
for seed in 0 1; do
  timeout -k 10 500 python3 -u scripts/iia_ceiling.py --model ioi-6l --epochs 1000 --every 50 --seed $seed --backend hip > $O/6l_s${seed}_hip_1000.log 2>&1 || { tail -20 $O/6l_s${seed}_hip_1000.log; exit 1; }
  grep -E '"metric"' $O/6l_s${seed}_hip_1000.log | cut -c1-400
done
