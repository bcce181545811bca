# Experiment: PyTorch TunableOp (exhaustive hipBLASLt/rocBLAS solution search per GEMM shape) for the library GEMMs.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tunableop
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop/results%d.csv
PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=20 timeout -k 10 700 python bench.py --steps 10 --warmup 3 > gpurun_out/tunableop/tune.log 2>&1 || { echo tune failed $?; tail -20 gpurun_out/tunableop/tune.log; exit 7; }
tail -1 gpurun_out/tunableop/tune.log
ls gpurun_out/tunableop
PYTORCH_TUNABLEOP_TUNING=0 IIT_GEMM_REPORT=gpurun_out/tunableop/gemm_decisions.txt timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/tunableop/use.log 2>&1 || { echo use failed $?; tail -20 gpurun_out/tunableop/use.log; exit 8; }
tail -1 gpurun_out/tunableop/use.log
