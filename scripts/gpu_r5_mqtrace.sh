set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5mq; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o mq -- python3 scripts/bench_families.py --family mqnli-bert-base --steps 12 --warmup 3 > $O/mq_prof.log 2>&1 || { tail -20 $O/mq_prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 8 --top 60 --gaps 8 > $O/mqnli_breakdown.txt && cat $O/mqnli_breakdown.txt | cut -c1-170; rm -rf $O/prof
