#!/bin/bash
# 6L/64d, seed 0, 160 epochs, fp32 torch-op backend: which bf16 rounding stops the model generalising?
#   f32: no rounding (control at this eval cadence); w: weights rounded to bf16 (straight-through gradient);
#   act: op outputs (and, through the casts, their gradients) rounded to bf16 (IIT_EMULATE_BF16, ops/torch_ops.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6z6
mkdir -p $O
for emu in none w act; do
  e=$emu; [ "$emu" = none ] && e=""
  IIT_EMULATE_BF16=$e timeout -k 10 420 python3 -u scripts/iia_ceiling.py --model ioi-6l --epochs 160 --every 40 --seed 0 \
    --backend torch > $O/$emu.log 2>&1 || { tail -20 $O/$emu.log; exit 1; }
  echo "== $emu"; grep -E '^Epoch (40|80|120|159):' $O/$emu.log | cut -c1-150
  grep -E '"metric"' $O/$emu.log | cut -c1-600
done
