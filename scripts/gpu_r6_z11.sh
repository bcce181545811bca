#!/bin/bash
# 6L/64d, seed 0, 160 epochs: the fp32 torch-op backend with BOTH weights and op outputs rounded to bf16
# (IIT_EMULATE_BF16=w,act; follow-up to gpu_r6_z6.sh, which rounded one or the other)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6z6
mkdir -p $O
IIT_EMULATE_BF16=w,act timeout -k 10 420 python3 -u scripts/iia_ceiling.py --model ioi-6l --epochs 160 --every 40 --seed 0 \
  --backend torch > $O/w_act.log 2>&1 || { tail -20 $O/w_act.log; exit 1; }
grep -E '^Epoch (40|80|120|159):' $O/w_act.log | cut -c1-150
grep -E '"metric"' $O/w_act.log | cut -c1-600
