set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5ht; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o b -- python3 bench.py --steps 15 --warmup 5 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 15 --top 45 --gaps 5 > $O/breakdown.txt && head -60 $O/breakdown.txt | cut -c1-170
rm -rf $O/prof
