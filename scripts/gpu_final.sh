# round-end rehearsal: GPU tests, smoke, and the driver's bench command
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_gpu.log; exit $rc; }
timeout -k 10 300 python __graft_entry__.py --smoke > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 3; }
tail -2 gpurun_out/smoke.log
IIT_GEMM_REPORT=gpurun_out/gemm_decisions.txt timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_final.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_final.log; exit 4; }
tail -1 gpurun_out/bench_final.log | cut -c1-300
grep -c " nan" gpurun_out/gemm_decisions.txt
