#!/bin/bash
# dual dX/dW cold-operand prefetch: tests, then headline A/B (IIT_DUAL_PREFETCH_WGS_PER_MB 0 = off / 4 / 8), same box
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6l
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_dual.py tests/test_headline_parity.py tests/test_paired.py -m gpu > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for k in 1 2; do
  for pf in 0 4 8; do
    timeout -k 10 200 env IIT_DUAL_PREFETCH_WGS_PER_MB=$pf python3 -u bench.py --gpus 1 --steps 40 --warmup 5 > $O/b_pf$pf.$k.log 2>&1 || { echo bench $pf failed; tail -20 $O/b_pf$pf.$k.log; exit 1; }
    echo "prefetch wgs/MB=$pf: $(grep -E '^\{' $O/b_pf$pf.$k.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
