#!/bin/bash
# round-6 final validation: GPU tests, smoke, the driver's bench command, and a graph-mode kernel trace of the headline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6final
mkdir -p $O
bash scripts/gpu_final.sh || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o hb -- python3 bench.py --gpus 1 --steps 10 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 8 --top 40 --gaps 5 > $O/headline_breakdown.txt && head -55 $O/headline_breakdown.txt; rm -f "$f"
