#!/bin/bash
# precision study, third seed: 6L/64d seed 2 -- HIP bf16 for the reference's 1000 epochs, fp32 oracle for 400
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6z14
mkdir -p $O
timeout -k 10 400 python3 -u scripts/iia_ceiling.py --model ioi-6l --epochs 1000 --every 100 --seed 2 --backend hip > $O/6l_s2_hip_1000.log 2>&1 || { tail -20 $O/6l_s2_hip_1000.log; exit 1; }
echo "== hip"; grep -E '^Epoch (50|100|200|300|400|600|800|999):' $O/6l_s2_hip_1000.log | cut -c1-150
timeout -k 10 640 python3 -u scripts/iia_ceiling.py --model ioi-6l --epochs 400 --every 100 --seed 2 --backend torch > $O/6l_s2_torch_400.log 2>&1 || { tail -20 $O/6l_s2_torch_400.log; exit 1; }
echo "== torch"; grep -E '^Epoch (50|100|200|300|399):' $O/6l_s2_torch_400.log | cut -c1-150
