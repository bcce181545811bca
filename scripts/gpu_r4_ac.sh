# Round 4 (session 2): position-major embedding backward (runs of equal tokens summed in registers): kernel tests, the
# full GPU suite, same-box A/B against the token-major kernel (IIT_EMBED_BWD_POS=0), two alternating rounds.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4ac
mkdir -p $O
j() { grep -E '^\{' $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "pairs/s", d["ms_per_step"], "ms")'; }
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 $O/tests.log)"; [ $rc -eq 0 ] || { grep -E "^FAILED" $O/tests.log | head; exit $rc; }
run() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py > $O/$name.log 2>&1 || { tail -20 $O/$name.log; exit 1; }
  echo "$name: $(j $name)"
}
for r in a b; do
  run pos_$r IIT_EMBED_BWD_POS=1
  run tok_$r IIT_EMBED_BWD_POS=0
done
