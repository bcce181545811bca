# GPU tests, the headline step breakdown at HEAD, and a roctx-marked (IIT_PROFILE=1) training run
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/stepprof gpurun_out/roctx
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/stepprof -o st -- \
  python3 bench.py --steps 20 --warmup 3 > gpurun_out/stepprof/bench.log 2>&1
rc=$?
echo "rocprof rc=$rc"
[ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/stepprof -name "*kernel_trace.csv" | head -n 1)
python scripts/step_breakdown.py "$f" --steps 15 --top 40 --gaps 6 --dump-step gpurun_out/stepprof/one_step.txt > gpurun_out/stepprof/breakdown.txt && head -3 gpurun_out/stepprof/breakdown.txt
rm -f "$f"
IIT_PROFILE=1 timeout -k 10 600 rocprofv3 --marker-trace --output-format csv -d gpurun_out/roctx -o tr -- \
  python3 scripts/time_to_iia.py --model gpt2-small --dtype bf16 --epochs 3 --num-samples 4000 > gpurun_out/roctx/train.log 2>&1
rc=$?
echo "marker rocprof rc=$rc"
[ $rc -eq 0 ] || exit $rc
m=$(find gpurun_out/roctx -name "*marker_api_trace.csv" | head -n 1)
python scripts/marker_summary.py "$m" > gpurun_out/roctx/summary.txt && head -25 gpurun_out/roctx/summary.txt
grep "\[perf\]" gpurun_out/roctx/train.log
rm -f "$m"
