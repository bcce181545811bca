# Round 4 (session 2): attention kernels with the spec path compiled out of the default instantiation, Adam unroll 4:
# GPU tests, bench x2, step breakdown.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4ab
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
step bench_a 300 python3 -u bench.py; j bench_a
step bench_b 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5; j bench_b
step prof 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o b -- python3 bench.py --steps 20 --warmup 3
f=$(find $O/prof -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 15 --top 40 --gaps 5 > $O/step_breakdown.txt && head -20 $O/step_breakdown.txt
rm -rf $O/prof
