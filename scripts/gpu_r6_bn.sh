#!/bin/bash
# conv reduction split-K (tests + per-layer timing); BN grid sizing A/B (IIT_BN_ROWS: 8 = round-5 default, 0 = target-grid sizing, 2 / 4 fixed), per layer and in the
# PVR bf16 step; after the BN tests (pivots kept in LDS for the finalize)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6bn
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bn_fused.py tests/test_conv_nhwc.py -m gpu > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 -u scripts/bench_conv.py > $O/conv.log 2>&1 || { echo bench_conv failed; tail -20 $O/conv.log; exit 1; }
cat $O/conv.log
for r in 8 0 2 4; do
  timeout -k 10 200 env IIT_BN_ROWS=$r python3 -u scripts/bench_bn.py > $O/bn_rows$r.log 2>&1 || { echo bench_bn $r failed; tail -20 $O/bn_rows$r.log; exit 1; }
  echo "rows=$r"; cat $O/bn_rows$r.log | grep layer
done
for k in 1 2; do
  for r in 8 0; do
    timeout -k 10 300 env IIT_BN_ROWS=$r python3 -u scripts/bench_families.py --family pvr-resnet18 --dtype bf16 --steps 30 --warmup 5 > $O/pvr_rows$r.$k.log 2>&1 || { echo pvr $r failed; tail -20 $O/pvr_rows$r.$k.log; exit 1; }
    echo "pvr rows=$r: $(grep -E '^\{' $O/pvr_rows$r.$k.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
