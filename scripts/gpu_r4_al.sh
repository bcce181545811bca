# Round 4 (session 2): full GPU suite + smoke + driver-default bench at the final HEAD
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4al
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu_tests rc=$rc"; tail -1 $O/gpu_tests.log; [ $rc -eq 0 ] || { tail -30 $O/gpu_tests.log; exit $rc; }
timeout -k 10 300 python3 -u __graft_entry__.py --smoke > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -E '^\{' $O/bench.log | cut -c1-400
