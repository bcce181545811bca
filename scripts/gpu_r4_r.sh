# Round 4 (session 2): eval sweeps after the one-capture prefix fix (official eval_ioi.py timing + profile), and the
# call sites of the Llama family's remaining elementwise kernels.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4r
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -30 $O/$name.log; exit $rc; fi
  return 0
}
step tests 300 python3 -u -m pytest tests/test_eval_ablations.py tests/test_eval_graphs_gpu.py -q -m gpu --timeout 120 --timeout-method thread
tail -1 $O/tests.log
step eval_profile 600 python3 -u scripts/profile_eval.py
grep -E "^\[eval\]" $O/eval_profile.log
step ioi_ckpt 300 python3 -u train_ioi.py --model gpt2-small --dtype bf16 --epochs 2 --num-samples 4000 --save-root /tmp/r4models --no-early-stop
step eval_ioi 600 python3 -u eval_ioi.py --model gpt2-small -w 100_100_40 --root /tmp/r4models --backend hip --num-samples 4608 --timing-repeats 2
grep -E "eval_ioi_timing" $O/eval_ioi.log | cut -c1-400
cp /tmp/r4models/IOI_ModelPair/100_100_40/results/results.csv $O/results.csv
step ops 600 python3 -u scripts/profile_family_ops.py --family llama-tiny-causal --seq 512
head -80 $O/ops.log
