set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3f
timeout -k 10 600 python3 -u -m pytest tests/test_paired.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3f/paired_tests.log 2>&1
rc=$?; tail -30 gpurun_out/r3f/paired_tests.log; echo "rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > gpurun_out/r3f/bench_paired.log 2>&1
rc=$?; grep -E '^\{' gpurun_out/r3f/bench_paired.log | cut -c1-300; echo "rc=$rc"
[ $rc -eq 0 ] || exit $rc
IIT_PAIRED=0 timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > gpurun_out/r3f/bench_unpaired.log 2>&1
rc=$?; grep -E '^\{' gpurun_out/r3f/bench_unpaired.log | cut -c1-300; echo "rc=$rc"
