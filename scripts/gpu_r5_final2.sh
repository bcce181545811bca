# round-5 late validation: GPU tests, smoke, driver bench, then the Llama-3-8B S=512 kernel breakdown (no splice passes)
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_final.sh || exit $?
mkdir -p gpurun_out/r5f
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5f/llprof -o ll -- python3 scripts/bench_families.py \
  --family llama3-8b-causal --seq 512 --steps 3 --warmup 2 > gpurun_out/r5f/llama_prof.log 2>&1 \
  || { echo "llama trace failed"; tail -20 gpurun_out/r5f/llama_prof.log; exit 1; }
grep -E '^\{' gpurun_out/r5f/llama_prof.log | cut -c1-200
f=$(find gpurun_out/r5f/llprof -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 3 --per-step-adam 3 --top 60 > gpurun_out/r5f/llama_breakdown.txt \
  && head -8 gpurun_out/r5f/llama_breakdown.txt; echo "splice rows: $(grep -c splice_kernel gpurun_out/r5f/llama_breakdown.txt)"; rm -f "$f"
