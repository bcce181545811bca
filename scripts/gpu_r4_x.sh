# Round 4 (session 2): same-box A/B of launch knobs at HEAD (driver-default bench): Adam unroll (U = 1 / 2 / 4), Adam
# non-temporal streams off, the GEMM XCD-local tile-order group height (4 / 8 / 16), two alternating rounds.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4x
mkdir -p $O
j() { grep -E '^\{' $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "pairs/s", d["ms_per_step"], "ms")'; }
run() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py > $O/$name.log 2>&1 || { tail -20 $O/$name.log; exit 1; }
  echo "$name: $(j $name)"
}
for r in a b; do
  run default_$r IIT_NOOP=1
  run adam_u4_$r IIT_ADAM_UNROLL=4
  run adam_u1_$r IIT_ADAM_UNROLL=1
  run adam_nt0_$r IIT_ADAM_NT=0
  run group4_$r IIT_GEMM_GROUP_M=4
  run group16_$r IIT_GEMM_GROUP_M=16
done
