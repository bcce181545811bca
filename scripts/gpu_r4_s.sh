# Round 4 (session 2): Llama torch backend with the bias in the projection GEMMs' epilogue (addmm) and the bias
# gradients from the weight-gradient GEMMs; tests, S=512 bench, kernel breakdown.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4s
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -30 $O/$name.log; exit $rc; fi
  return 0
}
jf() { grep -E '^\{' $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], d["ms_per_step"], "ms", "peak", d.get("peak_mem_gb"))'; }
step tests 300 python3 -u -m pytest tests/test_llama_ops.py tests/test_fused_norm.py -q -m gpu --timeout 120 --timeout-method thread
tail -1 $O/tests.log
F="scripts/bench_families.py --family llama3-8b-causal --seq 512 --steps 4 --warmup 2"
step ll_new 600 python3 -u $F; jf ll_new
step ll_prof 900 rocprofv3 --kernel-trace --output-format csv -d $O/llprof -o ll -- python3 $F
f=$(find $O/llprof -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 3 --top 40 --gaps 3 > $O/llama_breakdown.txt && head -40 $O/llama_breakdown.txt
rm -rf $O/llprof
