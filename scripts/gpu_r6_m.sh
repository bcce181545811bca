#!/bin/bash
# dual probe with the perfect-prefetch condition (evict_read) + prefetch density 8 / 16 / 32 per MiB A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6m
mkdir -p $O
timeout -k 10 300 python3 -u scripts/dual_l2_probe.py > $O/time.log 2>&1 || { echo probe failed; tail -20 $O/time.log; exit 1; }
tail -12 $O/time.log
for k in 1 2; do
  for pf in 0 8 16 32; do
    timeout -k 10 200 env IIT_DUAL_PREFETCH_WGS_PER_MB=$pf python3 -u bench.py --gpus 1 --steps 40 --warmup 5 > $O/b_pf$pf.$k.log 2>&1 || { echo bench $pf failed; tail -20 $O/b_pf$pf.$k.log; exit 1; }
    echo "prefetch wgs/MB=$pf: $(grep -E '^\{' $O/b_pf$pf.$k.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
