# Round 4 (session 2): paired-forward splice tests (hook_post inside the W_in op), then the dual kernels' tile-order
# group height A/B (IIT_GEMM_DUAL_GROUP_M; single launches at the new default 4), two alternating rounds.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4y
mkdir -p $O
j() { grep -E '^\{' $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "pairs/s", d["ms_per_step"], "ms")'; }
timeout -k 10 400 python3 -u -m pytest tests/test_paired.py tests/test_splice.py tests/test_hip_model.py tests/test_ioi_and_pairs.py -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 $O/tests.log)"; [ $rc -eq 0 ] || { grep -E "^FAILED|Error" $O/tests.log | head; exit $rc; }
run() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py > $O/$name.log 2>&1 || { tail -20 $O/$name.log; exit 1; }
  echo "$name: $(j $name)"
}
for r in a b; do
  run default_$r IIT_NOOP=1
  run dual4_$r IIT_GEMM_DUAL_GROUP_M=4
  run dual2_$r IIT_GEMM_DUAL_GROUP_M=2
  run dual16_$r IIT_GEMM_DUAL_GROUP_M=16
  run single8_$r IIT_GEMM_GROUP_M=8
done
