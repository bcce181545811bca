#!/bin/bash
# validation at HEAD: GPU tests, smoke, driver bench, headline kernel breakdown, PVR default vs library-only (same box)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6q
mkdir -p $O
bash scripts/gpu_final.sh || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o hb -- python3 bench.py --gpus 1 --steps 10 --warmup 3 --graphs 0 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 6 --top 30 --gaps 5 > $O/headline_breakdown.txt && head -40 $O/headline_breakdown.txt; rm -f "$f"
for k in 1 2; do
  for cfg in "IIT_CONV_HIP=auto" "IIT_CONV_HIP=0"; do
    timeout -k 10 300 env $cfg python3 -u scripts/bench_families.py --family pvr-resnet18 --dtype bf16 --steps 30 --warmup 5 > $O/pvr_$cfg.$k.log 2>&1 || { echo pvr failed; tail -20 $O/pvr_$cfg.$k.log; exit 1; }
    echo "pvr $cfg: $(grep -E '^\{' $O/pvr_$cfg.$k.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
