#!/bin/bash
# Round 5: fused BN (+res) (+ReLU) tests, PVR family step fused vs module path, kernel breakdown of the fused bf16 step
set -o pipefail
O=gpurun_out/r5i; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest tests/test_bn_fused.py -q -x --timeout 120 --timeout-method thread > $O/bn.log 2>&1 || { tail -40 $O/bn.log; exit 1; }
tail -2 $O/bn.log
for v in 0 1; do
  IIT_FUSED_BN=$v timeout -k 10 400 python3 -u scripts/bench_families.py --family pvr-resnet18 --dtype bf16 --steps 20 --warmup 3 > $O/fam_pvr_bf16_fused$v.log 2>&1 || { tail -20 $O/fam_pvr_bf16_fused$v.log; exit 1; }
  echo "fused=$v"; grep -E '^\{' $O/fam_pvr_bf16_fused$v.log | cut -c1-220
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/pvrprof -o pvr -- python3 scripts/bench_families.py --family pvr-resnet18 --dtype bf16 --steps 10 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/pvrprof -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 6 --top 30 --gaps 3 > $O/pvr_bf16_breakdown.txt && head -40 $O/pvr_bf16_breakdown.txt; rm -f "$f"
