# Round 3 batch 9: Llama-3-8B weight gradients through the GEMM dispatcher (LDS-DMA fp32-store/accumulate vs
# hipBLASLt per shape): GPU tests, S=512 family bench, steady-state step breakdown.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3k
run() {
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/r3k/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; grep -v amdgpu.ids "gpurun_out/r3k/$name.log" | grep -vE '^[EW]2026' | tail -3 | cut -c1-600
  if [ $rc -ge 124 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
  return 0
}
run tests 600 python3 -u -m pytest tests/test_llama_ops.py tests/test_causal_graph.py tests/test_flat_arena.py tests/test_gemm_dispatch.py -x -q -m gpu --timeout 300 --timeout-method thread
run llama_s512 900 python3 -u scripts/bench_families.py --family llama3-8b-causal --seq 512 --steps 4 --warmup 2
run llama_trace 900 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3k/ll -o ll -- python3 -u scripts/bench_families.py --family llama3-8b-causal --seq 512 --steps 4 --warmup 2
f=$(find gpurun_out/r3k/ll -name "*kernel_trace.csv" | head -n 1)
python3 scripts/step_breakdown.py "$f" --steps 3 --per-step-adam 3 --top 30 > gpurun_out/r3k/llama_step_breakdown.txt; rm -f "$f"
echo "batch done"
