set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5pt32; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o pv -- python3 scripts/bench_families.py --family pvr-resnet18 --dtype fp32 --steps 10 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 6 --top 45 --gaps 5 > $O/breakdown.txt && cat $O/breakdown.txt | cut -c1-160; rm -rf $O/prof
