# Round 4 (session 2): eval-sweep GEMM shapes into the shipped table (cold eval without autotune), cold eval_ioi with
# the extended table, and the 2-rank data-parallel rehearsal (gloo, one GPU) of the headline bench, replicated and
# ZeRO-1.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4u
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -30 $O/$name.log; exit $rc; fi
  return 0
}
step paired_tests 400 python3 -u -m pytest tests/test_paired.py tests/test_splice.py tests/test_hip_model.py -q -m gpu --timeout 120 --timeout-method thread
tail -1 $O/paired_tests.log
step tune_eval 600 python3 -u scripts/tune_eval_shapes.py --out $O/table_with_eval.json
grep tune-eval $O/tune_eval.log
step ioi_ckpt 300 python3 -u train_ioi.py --model gpt2-small --dtype bf16 --epochs 2 --num-samples 4000 --save-root /tmp/r4models --no-early-stop
IIT_GEMM_TABLE=$O/table_with_eval.json step eval_cold 600 python3 -u eval_ioi.py --model gpt2-small -w 100_100_40 --root /tmp/r4models --backend hip --num-samples 4608 --timing-repeats 2
grep -E "eval_ioi_timing" $O/eval_cold.log | cut -c1-400
export IIT_REHEARSE_ONE_GPU=1 IIT_DIST_BACKEND=gloo
step dp2 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 4 --warmup 3
grep -E '^\{' $O/dp2.log | cut -c1-250
IIT_ZERO=1 step dp2_zero 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 4 --warmup 3
grep -E '^\{' $O/dp2_zero.log | cut -c1-250
