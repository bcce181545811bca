#!/bin/bash
# 6L/64d plateau exit, long runs: fp32 torch-op oracle 700 epochs (seed 0); the HIP bf16 run follows in gpu_r6_z2.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6z
mkdir -p $O
timeout -k 10 1100 python3 -u scripts/iia_ceiling.py --model ioi-6l --epochs 700 --every 50 --seed 0 --backend torch > $O/6l_s0_torch_700.log 2>&1 || { tail -20 $O/6l_s0_torch_700.log; exit 1; }
grep -E '"metric"' $O/6l_s0_torch_700.log | cut -c1-400
