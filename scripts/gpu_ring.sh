set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_glds.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_glds.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_glds.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_glds.log; exit $rc; }
timeout -k 10 300 python -u scripts/bench_ring_depth.py > gpurun_out/ring_depth.txt 2>&1
rc=$?; cat gpurun_out/ring_depth.txt; [ $rc -eq 0 ] || exit $rc
IIT_GEMM_REPORT=gpurun_out/gemm_decisions.txt timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_native.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_native.log; exit 5; }
tail -1 gpurun_out/bench_native.log | cut -c1-250
