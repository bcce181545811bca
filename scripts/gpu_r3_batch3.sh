# Round 3 batch 3: epilogue store flavour A/B inside the real step, headline step breakdown (in-context table),
# PVR / Llama S=512 steady-state step breakdowns, IOI duplicate-node learnability probe.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3c
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/r3c/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; grep -v amdgpu.ids "gpurun_out/r3c/$name.log" | grep -vE '^[EW]2026' | tail -3 | cut -c1-600
  if [ $rc -ge 124 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
  return 0
}
for sm in 0 1 2 0; do
  IIT_GEMM_STORE=$sm run bench_store$sm 300 python3 -u bench.py --steps 100 --warmup 10
done
run step_prof 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3c/st -o st -- python3 -u bench.py --steps 30 --warmup 5
f=$(find gpurun_out/r3c/st -name "*kernel_trace.csv" | head -n 1)
python3 scripts/step_breakdown.py "$f" --steps 25 --top 45 --gaps 6 > gpurun_out/r3c/step_breakdown.txt; rm -f "$f"
run pvr_trace 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3c/pv -o pv -- python3 -u scripts/bench_families.py --family pvr-resnet18 --steps 40 --warmup 5
f=$(find gpurun_out/r3c/pv -name "*kernel_trace.csv" | head -n 1)
python3 scripts/step_breakdown.py "$f" --steps 30 --per-step-adam 2 --top 30 > gpurun_out/r3c/pvr_step_breakdown.txt; rm -f "$f"
run llama_trace 900 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3c/ll -o ll -- python3 -u scripts/bench_families.py --family llama3-8b-causal --seq 512 --steps 4 --warmup 1
f=$(find gpurun_out/r3c/ll -name "*kernel_trace.csv" | head -n 1)
python3 scripts/step_breakdown.py "$f" --steps 3 --per-step-adam 3 --top 30 > gpurun_out/r3c/llama_step_breakdown.txt; rm -f "$f"
run dup_probe 500 python3 -u scripts/iia_ceiling.py --epochs 25 --every 5 --train-nodes hook_duplicate
echo "batch done"
