# Round 4: headline A/B (default, no s+hip split-store candidate, no library GEMM at all), kernel trace of the headline
# step, PMC pass (MFMA busy), DP schedule breakdown at world 1 (replicated + ZeRO-1).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4g
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then tail -20 $O/$name.log; exit $rc; fi
  return 0
}
j() { grep -E '^\{' $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "pairs/s", d["ms_per_step"], "ms")'; }
IIT_CHECK_BOUNDS=1 step poison_bounds 300 python3 -u scripts/diag_uninit_poison.py --focused; grep -E "^\[bisect\]|Error" $O/poison_bounds.log | cut -c1-300
step ln_tests 300 python3 -u -m pytest tests/test_hip_kernels.py tests/test_hip_model.py -q -m gpu -k "layernorm or bert or mqnli" --timeout 120 --timeout-method thread; tail -2 $O/ln_tests.log
IIT_BERT_PAIRED=1 step fam_mqnli 400 python3 -u scripts/bench_families.py --family mqnli-bert-base --steps 30 --warmup 5; grep -E '^\{' $O/fam_mqnli.log | cut -c1-200
IIT_BERT_PAIRED=1 step fam_mqnli_prof 400 rocprofv3 --kernel-trace --output-format csv -d $O/mqprof -o mq -- python3 scripts/bench_families.py --family mqnli-bert-base --steps 20 --warmup 5
f=$(find $O/mqprof -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 12 --top 30 --gaps 5 > $O/mqnli_breakdown.txt && head -30 $O/mqnli_breakdown.txt; rm -f "$f"
step bench_default 300 python3 -u bench.py; j bench_default
IIT_GEMM_EXCLUDE='s\+hip' step bench_nosplitstore 300 python3 -u bench.py; j bench_nosplitstore
IIT_GEMM_EXCLUDE='blas.*' step bench_nolib 300 python3 -u bench.py; j bench_nolib
step bench_default2 300 python3 -u bench.py; j bench_default2
step prof 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o st -- python3 bench.py --steps 20 --warmup 3
f=$(find $O/prof -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 15 --top 45 --gaps 6 > $O/step_breakdown.txt && head -60 $O/step_breakdown.txt; rm -f "$f"
IIT_GEMM_EXCLUDE='blas.*' step prof_nolib 400 rocprofv3 --kernel-trace --output-format csv -d $O/profnl -o st -- python3 bench.py --steps 20 --warmup 3
f=$(find $O/profnl -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 15 --top 45 --gaps 6 > $O/step_breakdown_nolib.txt && head -30 $O/step_breakdown_nolib.txt; rm -f "$f"
for z in 0 1; do
  IIT_ZERO=$z RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=2954$z IIT_DP_FORCE_REDUCER=1 \
    step dp_prof_z$z 400 rocprofv3 --kernel-trace --output-format csv -d $O/dpprof$z -o dp -- python3 bench.py --steps 20 --warmup 3
  f=$(find $O/dpprof$z -name "*kernel_trace.csv" | head -n 1)
  [ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 15 --top 40 --gaps 12 > $O/dp_breakdown_z$z.txt && head -40 $O/dp_breakdown_z$z.txt; rm -f "$f"
done
