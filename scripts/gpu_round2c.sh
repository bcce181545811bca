# GEMM tests (shared split-K workspace), the 2-rank DP rehearsal on one GPU, the one-rank RCCL DP schedule profile,
# and the headline bench
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_glds.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_glds.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_glds.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_dp_rehearsal.sh || exit $?
bash scripts/gpu_dp_profile.sh > gpurun_out/dp_profile.out 2>&1
rc=$?; head -4 gpurun_out/dp_profile.out; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_native.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_native.log; exit 5; }
tail -1 gpurun_out/bench_native.log | cut -c1-250
