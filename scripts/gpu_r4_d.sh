# Round 4, validation + measurements of the opt-in features: BERT paired (+ LN splice), Llama residual epilogue /
# RMS fork, graphed eval sweeps, graph priming (time to IIA), DP schedule at world 1, PVR eval scripts.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4d
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then tail -20 $O/$name.log; exit $rc; fi
  return 0
}
step feat_tests 600 python3 -u -m pytest tests/test_hip_model.py tests/test_llama_ops.py tests/test_paired.py tests/test_dp_rccl_gpu.py -q -m gpu --timeout 300 --timeout-method thread
tail -3 $O/feat_tests.log; grep -E "^FAILED|^ERROR" $O/feat_tests.log | head
IIT_BERT_PAIRED=0 step fam_mqnli_off 400 python3 -u scripts/bench_families.py --family mqnli-bert-base --steps 30 --warmup 5; grep -E '^\{' $O/fam_mqnli_off.log | cut -c1-200
IIT_BERT_PAIRED=1 step fam_mqnli_on 400 python3 -u scripts/bench_families.py --family mqnli-bert-base --steps 30 --warmup 5; grep -E '^\{' $O/fam_mqnli_on.log | cut -c1-200
IIT_BERT_PAIRED=1 step fam_mqnli_prof 400 rocprofv3 --kernel-trace --output-format csv -d $O/mqprof -o mq -- python3 scripts/bench_families.py --family mqnli-bert-base --steps 12 --warmup 3
f=$(find $O/mqprof -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 8 --top 30 --gaps 5 > $O/mqnli_breakdown.txt && head -36 $O/mqnli_breakdown.txt; rm -f "$f"
for z in 0 1; do
  IIT_ZERO=$z RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=2953$z IIT_DP_FORCE_REDUCER=1 \
    step dp_bench_z$z 300 python3 -u bench.py --steps 30 --warmup 5; grep -E '^\{' $O/dp_bench_z$z.log | cut -c1-160
done
step ioi_ckpt 300 python3 -u train_ioi.py --model gpt2-small --dtype bf16 --epochs 2 --num-samples 4000 --save-root /tmp/r4models --no-early-stop
IIT_EVAL_GRAPHS=0 step eval_ioi_eager 600 python3 -u eval_ioi.py --model gpt2-small -w 100_100_40 --root /tmp/r4models --backend hip --num-samples 4608 --timing-repeats 2; grep -E "eval_ioi_timing" $O/eval_ioi_eager.log | cut -c1-400
IIT_EVAL_GRAPHS=1 step eval_ioi_graphs 600 python3 -u eval_ioi.py --model gpt2-small -w 100_100_40 --root /tmp/r4models --backend hip --num-samples 4608 --timing-repeats 2; grep -E "eval_ioi_timing" $O/eval_ioi_graphs.log | cut -c1-400
IIT_PROFILE=1 step tti_gpt2 500 python3 -u scripts/time_to_iia.py --model gpt2-small --dtype bf16 --epochs 80; grep -E "primed|^\{" $O/tti_gpt2.log | cut -c1-700
step eval_pvr 900 python3 -u scripts/eval_pvr_r4.py; grep -E "^\[pvr\]" $O/eval_pvr.log
step fam_pvr_fp32 400 python3 -u scripts/bench_families.py --family pvr-resnet18 --steps 20 --warmup 3; grep -E '^\{' $O/fam_pvr_fp32.log | cut -c1-200
step fam_pvr_bf16 400 python3 -u scripts/bench_families.py --family pvr-resnet18 --dtype bf16 --steps 20 --warmup 3; grep -E '^\{' $O/fam_pvr_bf16.log | cut -c1-200
step fam_pvr_bf16_prof 400 rocprofv3 --kernel-trace --output-format csv -d $O/pvrprof -o pvr -- python3 scripts/bench_families.py --family pvr-resnet18 --dtype bf16 --steps 10 --warmup 3
f=$(find $O/pvrprof -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 6 --top 25 --gaps 3 > $O/pvr_bf16_breakdown.txt && head -30 $O/pvr_bf16_breakdown.txt; rm -f "$f"
