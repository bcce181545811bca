# Round 4, first call: baseline bench on this box, overlapped-Adam GPU test + same-box A/B, cross-stream overlap probe,
# QKV-forward tile study, headline parity test.  Stops at the first crash / timeout (rc >= 124 or signal).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4a
mkdir -p $O
step() {  # step <name> <timeout> <cmd...>: log to $O/<name>.log; stop the call on a crash or timeout
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then tail -20 $O/$name.log; exit $rc; fi
  return 0
}
step bench_default 300 python3 -u bench.py; grep -E '^\{' $O/bench_default.log | cut -c1-200
IIT_ADAM_OVERLAP=1 step bench_overlap 300 python3 -u bench.py; grep -E '^\{' $O/bench_overlap.log | cut -c1-200
IIT_TEST_ADAM_OVERLAP=1 step adam_overlap_test 300 python3 -u -m pytest tests/test_adam_overlap.py -x -v -m gpu --timeout 120 --timeout-method thread; tail -4 $O/adam_overlap_test.log
step stream_overlap 200 python3 -u scripts/diag_stream_overlap.py; cat $O/stream_overlap.log
step qkv_fwd 200 python3 -u scripts/bench_qkv_fwd.py; cat $O/qkv_fwd.log
step headline_parity 600 python3 -u -m pytest tests/test_headline_parity.py -x -v -s -m gpu --timeout 500 --timeout-method thread; grep -E "grad norms|step losses|worst|passed|failed|Error|assert" $O/headline_parity.log | cut -c1-400
