#!/bin/bash
# PVR: which conv geometries pay in context (IIT_CONV_GEOMS A/B, decisions report); dual probe; prefetch density A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6o
mkdir -p $O
for k in 1 2; do
  for g in k3s1 k3s1,k3s2 k3s1,k1s2 k3s1,k3s2,k1s1,k1s2; do
    timeout -k 10 300 env IIT_CONV_GEOMS=$g IIT_CONV_REPORT=1 python3 -u scripts/bench_families.py --family pvr-resnet18 --dtype bf16 --steps 30 --warmup 5 > $O/pvr_$g.$k.log 2>&1 || { echo pvr failed; tail -20 $O/pvr_$g.$k.log; exit 1; }
    echo "pvr geoms=$g: $(grep -E '^\{' $O/pvr_$g.$k.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
grep -E "^(fwd|dgrad|wgrad)" "$O/pvr_k3s1,k3s2,k1s1,k1s2.1.log" | cut -c1-200
timeout -k 10 300 python3 -u scripts/dual_l2_probe.py > $O/time.log 2>&1 || { echo probe failed; tail -20 $O/time.log; exit 1; }
tail -9 $O/time.log
for k in 1 2; do
  for pf in 0 8 16 32; do
    timeout -k 10 200 env IIT_DUAL_PREFETCH_WGS_PER_MB=$pf python3 -u bench.py --gpus 1 --steps 40 --warmup 5 > $O/b_pf$pf.$k.log 2>&1 || { echo bench $pf failed; tail -20 $O/b_pf$pf.$k.log; exit 1; }
    echo "prefetch wgs/MB=$pf: $(grep -E '^\{' $O/b_pf$pf.$k.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
