#!/bin/bash
# transposed conv: per-shape in-place vs re-laid choice; tests + PVR vs library-only (same box) + decisions
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6v
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_nhwc.py tests/test_bn_fused.py tests/test_mnist_pvr_gpu.py -m gpu > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for k in 1 2; do
  for cfg in "IIT_CONV_HIP=auto" "IIT_CONV_HIP=0"; do
    timeout -k 10 300 env $cfg IIT_CONV_REPORT=1 python3 -u scripts/bench_families.py --family pvr-resnet18 --dtype bf16 --steps 30 --warmup 5 > $O/pvr_$cfg.$k.log 2>&1 || { echo pvr failed; tail -20 $O/pvr_$cfg.$k.log; exit 1; }
    echo "pvr $cfg: $(grep -E '^\{' $O/pvr_$cfg.$k.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
grep -E "^dgrad" "$O/pvr_IIT_CONV_HIP=auto.1.log" | cut -c1-170
