# Round 4 (session 2): Adam grid size A/B in the headline step (IIT_ADAM_MAX_BLOCKS: 4096 = the previous fixed grid,
# each workgroup striding over ~7 spans of 1024 float4 groups; larger = finer-grained hardware scheduling).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4z
mkdir -p $O
j() { grep -E '^\{' $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "pairs/s", d["ms_per_step"], "ms")'; }
run() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py > $O/$name.log 2>&1 || { tail -20 $O/$name.log; exit 1; }
  echo "$name: $(j $name)"
}
for r in a b; do
  run blocks4096_$r IIT_ADAM_MAX_BLOCKS=4096
  run blocks16384_$r IIT_ADAM_MAX_BLOCKS=16384
  run blocks65536_$r IIT_ADAM_MAX_BLOCKS=65536
  run blocks2048_$r IIT_ADAM_MAX_BLOCKS=2048
done
