#!/bin/bash
# 6L/64d IIA seeds x engines + reference-eager denominator; BN rows 16 / 32; PVR bf16 op sites
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6k
mkdir -p $O
for r in 16 32; do
  timeout -k 10 200 env IIT_BN_ROWS=$r python3 -u scripts/bench_bn.py > $O/bn_rows$r.log 2>&1 || { echo bench_bn $r failed; tail -20 $O/bn_rows$r.log; exit 1; }
  echo "rows=$r"; grep layer $O/bn_rows$r.log
done
timeout -k 10 300 python3 -u scripts/op_sites.py --family pvr-resnet18 --dtype bf16 > $O/pvr_sites.txt 2>&1 || { echo sites failed; tail -20 $O/pvr_sites.txt; exit 1; }
head -45 $O/pvr_sites.txt
bash scripts/gpu_r6_iia6l.sh
