#!/bin/bash
# LN backward rows per wave, MQNLI step: R = 1 vs the default 2, interleaved (follow-up to gpu_r6_z7.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6z8
mkdir -p $O
for r in 1 2 1 2 1 2; do
  IIT_LN_PART_R=$r timeout -k 10 300 python3 -u scripts/bench_families.py --family mqnli-bert-base --steps 30 --warmup 5 > $O/mq$r.log 2>&1 || { tail -20 $O/mq$r.log; exit 1; }
  echo "R=$r mqnli: $(grep -E '^\{' $O/mq$r.log | grep -oE '"ms_per_step": [0-9.]+')"
done
