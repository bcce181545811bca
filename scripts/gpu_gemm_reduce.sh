# reduction split-K: GEMM kernel tests, then the headline bench with the dispatcher's decisions recorded
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_glds.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_glds.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_glds.log
[ $rc -eq 0 ] || exit $rc
IIT_GEMM_REPORT=gpurun_out/gemm_decisions.txt timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_native.log 2>&1 || { echo bench failed $?; tail -30 gpurun_out/bench_native.log; exit 4; }
tail -1 gpurun_out/bench_native.log
grep "mode= 3" gpurun_out/gemm_decisions.txt | cut -c1-90
