set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3j
timeout -k 10 600 python3 -u -m pytest tests/test_paired.py tests/test_splice.py tests/test_hip_model.py tests/test_ioi_and_pairs.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r3j/tests.log 2>&1
rc=$?; tail -5 gpurun_out/r3j/tests.log; echo "rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > gpurun_out/r3j/bench.log 2>&1
rc=$?; grep -E '^\{' gpurun_out/r3j/bench.log | cut -c1-250; echo "rc=$rc"
