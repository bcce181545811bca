# Round 4 (session 2): validation of HEAD on a fresh build (GPU tests, smoke, bench) and the node-batched eval sweeps
# (IIT_EVAL_GROUP_ROWS=0: one spliced forward per node, the previous behaviour).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4n
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
step bench_a 300 python3 -u bench.py; j bench_a
step ioi_ckpt 300 python3 -u train_ioi.py --model gpt2-small --dtype bf16 --epochs 2 --num-samples 4000 --save-root /tmp/r4models --no-early-stop
IIT_EVAL_GROUP_ROWS=0 step eval_pernode 600 python3 -u eval_ioi.py --model gpt2-small -w 100_100_40 --root /tmp/r4models --backend hip --num-samples 4608 --timing-repeats 2
grep -E "eval_ioi_timing" $O/eval_pernode.log | cut -c1-400
cp /tmp/r4models/IOI_ModelPair/100_100_40/results/results.csv $O/results_pernode.csv
step eval_grouped 600 python3 -u eval_ioi.py --model gpt2-small -w 100_100_40 --root /tmp/r4models --backend hip --num-samples 4608 --timing-repeats 2
grep -E "eval_ioi_timing" $O/eval_grouped.log | cut -c1-400
cp /tmp/r4models/IOI_ModelPair/100_100_40/results/results.csv $O/results_grouped.csv
python3 - <<'EOF'
import csv
a = list(csv.DictReader(open("gpurun_out/r4n/results_pernode.csv")))
b = list(csv.DictReader(open("gpurun_out/r4n/results_grouped.csv")))
cols = [c for c in a[0] if c.endswith("effect")]
worst = 0.0
for x, y in zip(a, b):
    assert x["node"] == y["node"]
    for c in cols:
        worst = max(worst, abs(float(x[c]) - float(y[c])))
print(f"per-node vs grouped: {len(a)} nodes x {cols}: max |diff| {worst:.3g}")
EOF
step bench_b 300 python3 -u bench.py; j bench_b
