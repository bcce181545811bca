#!/bin/bash
# BatchNorm statistics from the conv epilogue: tests, PVR bf16 step A/B (IIT_BN_CONV_STATS 1 / 0), traced breakdown
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6i
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_nhwc.py tests/test_bn_fused.py tests/test_mnist_pvr_gpu.py -m gpu > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for k in 1 2; do
  for r in 1 0; do
    timeout -k 10 300 env IIT_BN_CONV_STATS=$r python3 -u scripts/bench_families.py --family pvr-resnet18 --dtype bf16 --steps 30 --warmup 5 > $O/pvr_cs$r.$k.log 2>&1 || { echo pvr $r failed; tail -20 $O/pvr_cs$r.$k.log; exit 1; }
    echo "pvr conv-stats=$r: $(grep -E '^\{' $O/pvr_cs$r.$k.log | grep -o '"ms_per_step": [0-9.]*\|"val_IIA": [0-9.]*' | tr '\n' ' ')"
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o pvr -- python3 scripts/bench_families.py --family pvr-resnet18 --dtype bf16 --steps 10 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 6 --top 45 --gaps 5 > $O/pvr_breakdown.txt && head -60 $O/pvr_breakdown.txt; rm -f "$f"
