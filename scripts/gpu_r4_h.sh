# Round 4: s+hip per-key bisect, graphed-eval / primed-training GPU tests, kernel stats of the eval sweep.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4h
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then tail -20 $O/$name.log; exit $rc; fi
  return 0
}
step keys 700 python3 -u scripts/diag_uninit_poison.py --keys; grep -E "^\[keys\]|^\[bisect\]" $O/keys.log | cut -c1-260
step eval_tests 600 python3 -u -m pytest tests/test_eval_graphs_gpu.py -v -m gpu --timeout 300 --timeout-method thread; grep -E "PASS|FAIL|Error|assert" $O/eval_tests.log | head -20
step ioi_ckpt 300 python3 -u train_ioi.py --model gpt2-small --dtype bf16 --epochs 2 --num-samples 4000 --save-root /tmp/r4models --no-early-stop
IIT_EVAL_GRAPHS=1 step eval_prof 600 rocprofv3 --kernel-trace --stats -d $O/evprof -o ev -- python3 eval_ioi.py --model gpt2-small -w 100_100_40 --root /tmp/r4models --backend hip --num-samples 4608 --timing-repeats 1
f=$(find $O/evprof -name "*kernel_stats.csv" | head -n 1)
[ -n "$f" ] && head -25 "$f" | cut -c1-220 > $O/eval_kernel_stats.txt && cat $O/eval_kernel_stats.txt
find $O/evprof -name "*kernel_trace.csv" -delete
