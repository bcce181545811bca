#!/bin/bash
# PVR: BatchNorm grid rows 8 (default) vs 16 vs 12, then 8 vs 6 vs 4 in the full step (forward and backward share the grid)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6y
mkdir -p $O
for k in 1 2; do
  for r in 8 6 4; do
    timeout -k 10 300 env IIT_BN_ROWS=$r python3 -u scripts/bench_families.py --family pvr-resnet18 --dtype bf16 --steps 30 --warmup 5 > $O/pvr_rows$r.$k.log 2>&1 || { echo pvr failed; tail -20 $O/pvr_rows$r.$k.log; exit 1; }
    echo "pvr rows=$r: $(grep -E '^\{' $O/pvr_rows$r.$k.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
