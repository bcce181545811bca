#!/bin/bash
# round-6 closing validation at HEAD: GPU tests, smoke, the driver's bench command; the bench with IIT_GEMM_FREEZE=1
# (every GEMM decision from the shipped table, no in-process timing); a kernel trace of the headline step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6final3
mkdir -p $O
bash scripts/gpu_final.sh || exit $?
IIT_GEMM_FREEZE=1 timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_freeze.log 2>&1 || { echo freeze bench failed; tail -20 $O/bench_freeze.log; exit 5; }
echo "freeze: $(tail -1 $O/bench_freeze.log | grep -oE '"ms_per_step": [0-9.]+')"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o hb -- python3 bench.py --gpus 1 --steps 10 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 8 --top 40 --gaps 5 > $O/headline_breakdown.txt && head -30 $O/headline_breakdown.txt; rm -f "$f"
