# Round 4 (session 2) final validation at HEAD (ragged tails on the repo kernels): every GPU test, smoke, the driver's bench command (twice), a kernel
# breakdown of the headline step and the in-step GEMM PMC summary (MFMA busy).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4aj
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -30 $O/$name.log; exit $rc; fi
  return 0
}
j() { grep -E '^\{' $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "pairs/s", d["ms_per_step"], "ms")'; }
step gpu_tests 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
tail -1 $O/gpu_tests.log
step smoke 300 python3 -u __graft_entry__.py --smoke
tail -1 $O/smoke.log | cut -c1-200
step bench_a 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5; j bench_a
step bench_b 300 python3 -u bench.py; j bench_b
step prof 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o b -- python3 bench.py --steps 20 --warmup 3
f=$(find $O/prof -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 15 --top 120 --gaps 5 > $O/step_breakdown.txt && head -30 $O/step_breakdown.txt && echo "Cijk rows: $(grep -c Cijk $O/step_breakdown.txt || true)"
rm -rf $O/prof
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc -o p -- python3 -u bench.py --graphs 0 --steps 6 --warmup 3 > $O/pmc_run.log 2>&1
rc=$?; echo "pmc rc=$rc"
[ $rc -eq 0 ] || exit $rc
f=$(find $O/pmc -name "*counter_collection.csv" | head -n 1)
python3 scripts/pmc_step_summary.py "$f" 4 > $O/pmc_step_summary.txt; tail -3 $O/pmc_step_summary.txt
rm -rf $O/pmc
export IIT_REHEARSE_ONE_GPU=1 IIT_DIST_BACKEND=gloo  # (ZeRO-1 rehearsals)
IIT_ZERO=1 step dp2_zero 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 4 --warmup 3
grep -E '^\{' $O/dp2_zero.log | cut -c1-200
unset IIT_REHEARSE_ONE_GPU IIT_DIST_BACKEND
IIT_ZERO=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29535 IIT_DP_FORCE_REDUCER=1 step dp1_zero 300 python3 -u bench.py --steps 30 --warmup 5
grep -E '^\{' $O/dp1_zero.log | cut -c1-200
