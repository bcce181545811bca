# Round 4: in-step GEMM counters (MFMA busy), Llama-3-8B S=512 family bench with the torch-backend fusions on / off and
# a kernel breakdown of the fused step.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4j
mkdir -p $O/pmc
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc -o p -- python3 -u bench.py --graphs 0 --steps 6 --warmup 3 > $O/pmc_run.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -2 $O/pmc_run.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
f=$(find $O/pmc -name "*counter_collection.csv" | head -n 1)
python3 scripts/pmc_step_summary.py "$f" 4 > $O/pmc_step_summary.txt; head -40 $O/pmc_step_summary.txt
rm -f $O/pmc/*.csv
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then tail -20 $O/$name.log; exit $rc; fi
  return 0
}
IIT_TORCH_RESID_EPI=0 IIT_RMS_FORK=0 step llama_off 500 python3 -u scripts/bench_families.py --family llama3-8b-causal --seq 512 --steps 5 --warmup 2; grep -E '^\{' $O/llama_off.log | cut -c1-260
IIT_TORCH_RESID_EPI=1 IIT_RMS_FORK=1 step llama_on 500 python3 -u scripts/bench_families.py --family llama3-8b-causal --seq 512 --steps 5 --warmup 2; grep -E '^\{' $O/llama_on.log | cut -c1-260
IIT_TORCH_RESID_EPI=1 IIT_RMS_FORK=1 step llama_prof 600 rocprofv3 --kernel-trace --output-format csv -d $O/llprof -o ll -- python3 scripts/bench_families.py --family llama3-8b-causal --seq 512 --steps 4 --warmup 2
f=$(find $O/llprof -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 3 --top 30 --gaps 3 > $O/llama_breakdown.txt && head -40 $O/llama_breakdown.txt; rm -f "$f"
