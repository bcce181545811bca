# GEMM kernel check on the GPU box: parity tests of the LDS-DMA GEMM, then the shape microbenchmark
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_glds.py tests/test_gemm_dispatch.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gemm.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gemm.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_gemm_glds.py > gpurun_out/gemm_glds_bench.txt 2>&1 || { echo bench failed; tail -20 gpurun_out/gemm_glds_bench.txt; exit 3; }
cat gpurun_out/gemm_glds_bench.txt
