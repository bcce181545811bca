# Kernel-level profile of the Llama-3-8B causal-graph family benchmark (1 GPU)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/llprof
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/llprof -o ll -- \
  python3 scripts/bench_families.py --family llama3-8b-causal --steps 3 --warmup 1 > gpurun_out/llprof/bench.log 2>&1
rc=$?
echo "rocprof rc=$rc"
tail -1 gpurun_out/llprof/bench.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/llprof -name "*kernel_stats.csv" | head -n 1)
python scripts/summarize_profile.py "$f" 4 40 > gpurun_out/llprof/top.txt && cat gpurun_out/llprof/top.txt
rm -f $(find gpurun_out/llprof -name "*kernel_trace.csv")
