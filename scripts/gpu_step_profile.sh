# Kernel trace of the headline bench (1 GPU) -> steady-state per-step breakdown with idle-gap attribution.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/stepprof
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/stepprof -o st -- \
  python3 bench.py --steps 20 --warmup 3 > gpurun_out/stepprof/bench.log 2>&1
rc=$?
echo "rocprof rc=$rc"
[ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/stepprof -name "*kernel_trace.csv" | head -n 1)
python scripts/step_breakdown.py "$f" --steps 15 --top 40 --gaps 6 --dump-step gpurun_out/stepprof/one_step.txt > gpurun_out/stepprof/breakdown.txt && cat gpurun_out/stepprof/breakdown.txt
rm -f "$f"
