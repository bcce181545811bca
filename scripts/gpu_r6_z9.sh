#!/bin/bash
# LN affine-gradient partial reduce: most groups G (IIT_LN_REDUCE_G = 32 default / 64 / 120), MQNLI step, interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6z9
mkdir -p $O
IIT_LN_REDUCE_G=120 timeout -k 10 300 python3 -u -m pytest tests/test_hip_kernels.py -k layernorm -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
echo "G=120 tests: $(tail -1 $O/t.log)"
for g in 32 64 120 32 64 120; do
  IIT_LN_REDUCE_G=$g timeout -k 10 300 python3 -u scripts/bench_families.py --family mqnli-bert-base --steps 30 --warmup 5 > $O/mq$g.log 2>&1 || { tail -20 $O/mq$g.log; exit 1; }
  echo "G=$g mqnli: $(grep -E '^\{' $O/mq$g.log | grep -oE '"ms_per_step": [0-9.]+')"
done
