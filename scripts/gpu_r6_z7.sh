#!/bin/bash
# LayerNorm backward with fused affine gradients: rows per wave (IIT_LN_PART_R = 1 / 2 / 4) -- numerics for each, then
# the MQNLI (BERT-base) step A/B, interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6z7
mkdir -p $O
for r in 1 2 4; do
  IIT_LN_PART_R=$r timeout -k 10 300 python3 -u -m pytest tests/test_hip_kernels.py -k layernorm -x -q --timeout 120 --timeout-method thread > $O/t$r.log 2>&1 || { tail -30 $O/t$r.log; exit 1; }
  echo "R=$r tests: $(tail -1 $O/t$r.log)"
done
for r in 2 4 1 2 4; do
  IIT_LN_PART_R=$r timeout -k 10 300 python3 -u scripts/bench_families.py --family mqnli-bert-base --steps 30 --warmup 5 > $O/mq$r.log 2>&1 || { tail -20 $O/mq$r.log; exit 1; }
  echo "R=$r mqnli: $(grep -E '^\{' $O/mq$r.log | grep -oE '"ms_per_step": [0-9.]+')"
done
