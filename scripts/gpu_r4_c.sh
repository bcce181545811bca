# Round 4 combined call: full GPU suite (kernels changed: transposed-accumulator epilogue, LN row select, RMS fork),
# bench A/B (default / overlapped Adam), stream-overlap probe, QKV tile study, headline parity.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4c
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then tail -20 $O/$name.log; exit $rc; fi
  return 0
}
step gpu_tests 900 python3 -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread --deselect tests/test_headline_parity.py
tail -3 $O/gpu_tests.log; grep -E "^FAILED|^ERROR|Error" $O/gpu_tests.log | head -10
step bench_default 300 python3 -u bench.py; grep -E '^\{' $O/bench_default.log | cut -c1-200
step bench_default2 300 python3 -u bench.py; grep -E '^\{' $O/bench_default2.log | cut -c1-200
step stream_overlap 200 python3 -u scripts/diag_stream_overlap.py; cat $O/stream_overlap.log
step qkv_fwd 200 python3 -u scripts/bench_qkv_fwd.py; cat $O/qkv_fwd.log
step poison 300 python3 -u scripts/diag_uninit_poison.py; grep -E "MISMATCH|differ" $O/poison.log | head -30
step headline_parity 600 python3 -u -m pytest tests/test_headline_parity.py -x -v -s -m gpu --timeout 500 --timeout-method thread; grep -E "grad norms|step losses|worst|passed|failed|Error|assert" $O/headline_parity.log | cut -c1-400
