#!/bin/bash
# PVR: conv decision policy A/B (library margin 0.15 default / 0 = plain isolated choice / IIT_CONV_HIP=1 all repo kernels)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6p
mkdir -p $O
for k in 1 2; do
  for cfg in "IIT_CONV_LIB_MARGIN=0.15" "IIT_CONV_LIB_MARGIN=0" "IIT_CONV_HIP=1"; do
    timeout -k 10 300 env $cfg IIT_CONV_REPORT=1 python3 -u scripts/bench_families.py --family pvr-resnet18 --dtype bf16 --steps 30 --warmup 5 > $O/pvr_$cfg.$k.log 2>&1 || { echo pvr failed; tail -20 $O/pvr_$cfg.$k.log; exit 1; }
    echo "pvr $cfg: $(grep -E '^\{' $O/pvr_$cfg.$k.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
grep -E "^(fwd|dgrad|wgrad)" "$O/pvr_IIT_CONV_LIB_MARGIN=0.15.1.log" | cut -c1-160
