#!/bin/bash
# general conv kernels (3x3 / 1x1, stride 1 / 2): tests + PVR A/B; dual probe with evict_read; prefetch density A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6n
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_nhwc.py tests/test_bn_fused.py tests/test_mnist_pvr_gpu.py -m gpu > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for k in 1 2; do
  timeout -k 10 300 python3 -u scripts/bench_families.py --family pvr-resnet18 --dtype bf16 --steps 30 --warmup 5 > $O/pvr$k.log 2>&1 || { echo pvr failed; tail -20 $O/pvr$k.log; exit 1; }
  echo "pvr: $(grep -E '^\{' $O/pvr$k.log | grep -o '"ms_per_step": [0-9.]*\|"val_IIA": [0-9.]*' | tr '\n' ' ')"
done
timeout -k 10 300 python3 -u scripts/dual_l2_probe.py > $O/time.log 2>&1 || { echo probe failed; tail -20 $O/time.log; exit 1; }
tail -9 $O/time.log
for k in 1 2; do
  for pf in 0 8 16 32; do
    timeout -k 10 200 env IIT_DUAL_PREFETCH_WGS_PER_MB=$pf python3 -u bench.py --gpus 1 --steps 40 --warmup 5 > $O/b_pf$pf.$k.log 2>&1 || { echo bench $pf failed; tail -20 $O/b_pf$pf.$k.log; exit 1; }
    echo "prefetch wgs/MB=$pf: $(grep -E '^\{' $O/b_pf$pf.$k.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
