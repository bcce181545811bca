# Round 4 (session 2): Adam work unit A/B with one workgroup per span: span length (IIT_ADAM_SPAN4) and unroll
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4aa
mkdir -p $O
j() { grep -E '^\{' $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "pairs/s", d["ms_per_step"], "ms")'; }
run() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py > $O/$name.log 2>&1 || { tail -20 $O/$name.log; exit 1; }
  echo "$name: $(j $name)"
}
for r in a b; do
  run default_$r IIT_NOOP=1
  run u4_$r IIT_ADAM_UNROLL=4
  run span512_$r IIT_ADAM_SPAN4=512
  run span2048_$r IIT_ADAM_SPAN4=2048
  run span2048u4_$r IIT_ADAM_SPAN4=2048 IIT_ADAM_UNROLL=4
done
