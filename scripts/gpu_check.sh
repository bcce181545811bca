set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
python -c "import torch; print(torch.cuda.get_device_name(0))" > gpurun_out/dev.log 2>&1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python __graft_entry__.py --smoke > gpurun_out/smoke.log 2>&1 || { echo smoke failed $?; tail -20 gpurun_out/smoke.log; exit 3; }
tail -3 gpurun_out/smoke.log
IIT_GEMM_REPORT=gpurun_out/gemm_decisions.txt timeout -k 10 500 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_native.log 2>&1 || { echo bench failed $?; tail -30 gpurun_out/bench_native.log; exit 4; }
tail -2 gpurun_out/bench_native.log
