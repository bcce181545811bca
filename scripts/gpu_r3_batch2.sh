# Round 3 batch 2: IIA-ceiling history, GEMM store-flavour boundary test, PVR + Llama S=512 records with kernel stats.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3b
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/r3b/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; grep -v amdgpu.ids "gpurun_out/r3b/$name.log" | tail -4 | cut -c1-400
  if [ $rc -ge 124 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
  return 0
}
run store_modes 200 python3 -u scripts/diag_store_modes.py
run iia_ceiling 600 python3 -u scripts/iia_ceiling.py --epochs 70 --every 5
run pvr_prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3b/pvrprof -o pvr -- python3 -u scripts/bench_families.py --family pvr-resnet18 --steps 10 --warmup 3
rm -f gpurun_out/r3b/pvrprof/*kernel_trace.csv
run llama_s512_prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3b/llprof -o llama -- python3 -u scripts/bench_families.py --family llama3-8b-causal --seq 512 --steps 3 --warmup 1
rm -f gpurun_out/r3b/llprof/*kernel_trace.csv
echo "batch done"
