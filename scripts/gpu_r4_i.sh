# Round 4: validation of BERT embed / token-type / ZeRO world-1 alias + row skipping / dispatcher fix, s+hip per-key
# bisect, graphed + prefix-shared eval sweeps, headline all-own-GEMM A/B.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4i
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
step tests 600 python3 -u -m pytest tests/test_hip_model.py tests/test_dp_rccl_gpu.py tests/test_eval_graphs_gpu.py tests/test_hip_kernels.py -q -m gpu --timeout 300 --timeout-method thread
tail -3 $O/tests.log; grep -E "^FAILED|^ERROR" $O/tests.log | head
IIT_CHECK_BOUNDS=1 step poison_bounds 300 python3 -u scripts/diag_uninit_poison.py --focused; grep -E "^\[bisect\]|Error" $O/poison_bounds.log | cut -c1-300
step keys 600 python3 -u scripts/diag_uninit_poison.py --keys; grep -E "^\[keys\]|^\[bisect\]" $O/keys.log | cut -c1-300
IIT_BERT_PAIRED=1 step fam_mqnli 400 python3 -u scripts/bench_families.py --family mqnli-bert-base --steps 30 --warmup 5; grep -E '^\{' $O/fam_mqnli.log | cut -c1-200
IIT_ZERO=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 IIT_DP_FORCE_REDUCER=1 step dp_bench_z1 300 python3 -u bench.py --steps 30 --warmup 5; j dp_bench_z1
step bench_default 300 python3 -u bench.py; j bench_default
step adam_micro 300 python3 -u scripts/bench_adam.py; grep -E "NT=" $O/adam_micro.log
IIT_GEMM_EXCLUDE='blas.*' step bench_nolib 300 python3 -u bench.py; j bench_nolib
step ioi_ckpt 300 python3 -u train_ioi.py --model gpt2-small --dtype bf16 --epochs 2 --num-samples 4000 --save-root /tmp/r4models --no-early-stop
IIT_EVAL_GRAPHS=1 step eval_ioi_graphs 600 python3 -u eval_ioi.py --model gpt2-small -w 100_100_40 --root /tmp/r4models --backend hip --num-samples 4608 --timing-repeats 2; grep -E "eval_ioi_timing" $O/eval_ioi_graphs.log | cut -c1-400
IIT_EVAL_GRAPHS=1 step eval_prof 600 rocprofv3 --kernel-trace --stats -d $O/evprof -o ev -- python3 eval_ioi.py --model gpt2-small -w 100_100_40 --root /tmp/r4models --backend hip --num-samples 4608 --timing-repeats 1
f=$(find $O/evprof -name "*kernel_stats.csv" | head -n 1)
[ -n "$f" ] && head -25 "$f" | cut -c1-200 > $O/eval_kernel_stats.txt && cat $O/eval_kernel_stats.txt
find $O/evprof -name "*kernel_trace.csv" -delete
