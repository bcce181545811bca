#!/bin/bash
# transposed conv reading the forward weight in place: tests, per-layer timing, PVR vs library-only; MQNLI prefetch A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6u
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_nhwc.py tests/test_bn_fused.py tests/test_mnist_pvr_gpu.py -m gpu > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 -u scripts/bench_conv.py > $O/conv.log 2>&1 || { echo bench_conv failed; tail -20 $O/conv.log; exit 1; }
grep -o '"layer": "[a-z0-9]*"\|"dgrad": {[^}]*}' $O/conv.log | paste - -
for k in 1 2; do
  for cfg in "IIT_CONV_HIP=auto" "IIT_CONV_HIP=0"; do
    timeout -k 10 300 env $cfg python3 -u scripts/bench_families.py --family pvr-resnet18 --dtype bf16 --steps 30 --warmup 5 > $O/pvr_$cfg.$k.log 2>&1 || { echo pvr failed; tail -20 $O/pvr_$cfg.$k.log; exit 1; }
    echo "pvr $cfg: $(grep -E '^\{' $O/pvr_$cfg.$k.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
for k in 1 2; do
  for pf in 16 0; do
    timeout -k 10 300 env IIT_DUAL_PREFETCH_WGS_PER_MB=$pf python3 -u scripts/bench_families.py --family mqnli-bert-base --steps 30 --warmup 5 > $O/mq_pf$pf.$k.log 2>&1 || { echo mq failed; tail -20 $O/mq_pf$pf.$k.log; exit 1; }
    echo "mqnli prefetch=$pf: $(grep -E '^\{' $O/mq_pf$pf.$k.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
