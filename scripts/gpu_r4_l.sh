# Round 4: LN-xhat16 backward A/B, priming trajectory test, in-step GEMM counters, time to IIA of the reference 6L model.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4l
mkdir -p $O/pmc
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then tail -20 $O/$name.log; exit $rc; fi
  return 0
}
j() { grep -E '^\{' $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "pairs/s", d["ms_per_step"], "ms")'; }
step bench_xh1 300 python3 -u bench.py; j bench_xh1
IIT_LN_XHAT16=0 step bench_xh0 300 python3 -u bench.py; j bench_xh0
step bench_xh1b 300 python3 -u bench.py; j bench_xh1b
IIT_LN_XHAT16=0 step bench_xh0b 300 python3 -u bench.py; j bench_xh0b
step primed 400 python3 -u -m pytest tests/test_eval_graphs_gpu.py tests/test_headline_parity.py -q -m gpu --tb=short --timeout 300 --timeout-method thread; grep -E "^E |passed|failed" $O/primed.log | head -12
IIT_PROFILE=1 step tti_6l 400 python3 -u scripts/time_to_iia.py --model ioi-6l --dtype bf16 --epochs 150; grep -E "primed|^\{" $O/tti_6l.log | cut -c1-700
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc -o p -- python3 -u bench.py --graphs 0 --steps 6 --warmup 3 > $O/pmc_run.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -2 $O/pmc_run.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
f=$(find $O/pmc -name "*counter_collection.csv" | head -n 1)
python3 scripts/pmc_step_summary.py "$f" 4 > $O/pmc_step_summary.txt; head -40 $O/pmc_step_summary.txt
rm -rf $O/pmc
