# Round 4, second call: DP schedule breakdown at world 1 (replicated + ZeRO-1), BERT paired GPU test, eval sweeps
# (graphed), time-to-IIA with primed graphs, PVR eval scripts vs the oracle path.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4b
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then tail -20 $O/$name.log; exit $rc; fi
  return 0
}
step bert_paired 300 python3 -u -m pytest tests/test_hip_model.py -x -v -m gpu -k "bert" --timeout 120 --timeout-method thread; tail -5 $O/bert_paired.log
for z in 0 1; do
  IIT_ZERO=$z RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=2953$z IIT_DP_FORCE_REDUCER=1 \
    step dp_bench_z$z 300 python3 -u bench.py --steps 30 --warmup 5; grep -E '^\{' $O/dp_bench_z$z.log | cut -c1-160
done
RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29535 IIT_DP_FORCE_REDUCER=1 \
  step dp_prof 400 rocprofv3 --kernel-trace --output-format csv -d $O/dpprof -o dp -- python3 bench.py --steps 20 --warmup 3
f=$(find $O/dpprof -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 15 --top 40 --gaps 12 > $O/dp_breakdown.txt && head -60 $O/dp_breakdown.txt; rm -f "$f"
step ioi_ckpt 300 python3 -u train_ioi.py --model gpt2-small --dtype bf16 --epochs 2 --num-samples 4000 --save-root /tmp/r4models --no-early-stop
step eval_ioi_hip 600 python3 -u eval_ioi.py --model gpt2-small -w 100_100_40 --root /tmp/r4models --backend hip --num-samples 4608 --timing-repeats 2; grep -E "eval_ioi_timing" $O/eval_ioi_hip.log | cut -c1-400
IIT_PROFILE=1 step tti_gpt2 500 python3 -u scripts/time_to_iia.py --model gpt2-small --dtype bf16 --epochs 80; grep -E "primed|^\{" $O/tti_gpt2.log | cut -c1-600
step eval_pvr 900 python3 -u scripts/eval_pvr_r4.py; grep -E "^\[pvr\]" $O/eval_pvr.log
step llama_tests 300 python3 -u -m pytest tests/test_llama_ops.py -x -v -m gpu --timeout 120 --timeout-method thread; tail -3 $O/llama_tests.log
step dp_tests 400 python3 -u -m pytest tests/test_dp_rccl_gpu.py -x -v -m gpu --timeout 200 --timeout-method thread; tail -3 $O/dp_tests.log
IIT_GEMM_TABLE=0 IIT_GEMM_REPORT=$O/gemm_report_isolated.txt step gemm_autotune 600 python3 -u bench.py --steps 5 --warmup 2; grep -E '^\{' $O/gemm_autotune.log | cut -c1-200
step fam_mqnli 400 python3 -u scripts/bench_families.py --family mqnli-bert-base --steps 30 --warmup 5; grep -E '^\{' $O/fam_mqnli.log | cut -c1-250
step fam_mqnli_prof 400 rocprofv3 --kernel-trace --output-format csv -d $O/mqprof -o mq -- python3 scripts/bench_families.py --family mqnli-bert-base --steps 12 --warmup 3
f=$(find $O/mqprof -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 8 --top 30 --gaps 5 > $O/mqnli_breakdown.txt && head -40 $O/mqnli_breakdown.txt; rm -f "$f"
