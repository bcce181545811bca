# Kernel trace of the data-parallel schedule on ONE GPU (one-rank RCCL group, reducer forced on), launched
# without torchrun so rocprofv3 wraps the python process itself; then the steady-state step breakdown.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/dpprof
RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29531 IIT_DP_FORCE_REDUCER=1 \
  timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/dpprof -o dp -- \
  python3 bench.py --steps 20 --warmup 3 > gpurun_out/dpprof/bench.log 2>&1
rc=$?
echo "rocprof rc=$rc"
tail -1 gpurun_out/dpprof/bench.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/dpprof -name "*kernel_trace.csv" | head -n 1)
python scripts/step_breakdown.py "$f" --steps 15 --top 25 --gaps 15 > gpurun_out/dpprof/breakdown.txt && cat gpurun_out/dpprof/breakdown.txt
rm -f "$f"
