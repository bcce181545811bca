#!/bin/bash
# Round 5: PVR bf16 step with the conv-hook splice read by the fused BatchNorm; splice_kernel rows in its trace
set -o pipefail
O=gpurun_out/r5n; mkdir -p $O
for v in 1 0; do
  IIT_BN_SPLICE=$v timeout -k 10 400 python3 -u scripts/bench_families.py --family pvr-resnet18 --dtype bf16 --steps 20 --warmup 3 > $O/bf16_splice$v.log 2>&1 || { tail -20 $O/bf16_splice$v.log; exit 1; }
  echo "IIT_BN_SPLICE=$v: $(grep -E '^\{' $O/bf16_splice$v.log | cut -c1-200)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/pvrprof -o pvr -- python3 scripts/bench_families.py --family pvr-resnet18 --dtype bf16 --steps 10 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/pvrprof -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 6 --top 60 --gaps 3 > $O/pvr_bf16_breakdown.txt && head -8 $O/pvr_bf16_breakdown.txt && (grep -c splice_kernel $O/pvr_bf16_breakdown.txt || true); rm -f "$f"
