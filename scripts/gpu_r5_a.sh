# round 5: 8-phase GEMM numerics + race screen, then the isolated benchmark
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_8ph.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5a_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5a_tests.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/r5a_tests.log; exit $rc; }
timeout -k 10 600 python -u scripts/bench_gemm_8ph.py > gpurun_out/r5a_bench.log 2>&1
rc=$?; tail -16 gpurun_out/r5a_bench.log; exit $rc
