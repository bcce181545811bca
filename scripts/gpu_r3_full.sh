# Full GPU suite + smoke + default bench (what the driver runs at round end).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3p
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3p/gpu_tests.log 2>&1
rc=$?; tail -6 gpurun_out/r3p/gpu_tests.log; echo "tests rc=$rc"
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3p/smoke.log 2>&1
rc2=$?; tail -2 gpurun_out/r3p/smoke.log; echo "smoke rc=$rc2"
[ $rc2 -ge 124 ] && exit $rc2
timeout -k 10 300 python3 -u bench.py > gpurun_out/r3p/bench.log 2>&1
rc3=$?; grep -E '^\{' gpurun_out/r3p/bench.log | cut -c1-300; echo "bench rc=$rc3"
exit $rc
