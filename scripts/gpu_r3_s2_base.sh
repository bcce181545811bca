# Round 3 session 2 baseline: headline bench at HEAD + kernel-trace step breakdown.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3s2a
timeout -k 10 300 python3 -u bench.py > gpurun_out/r3s2a/bench_default.log 2>&1 || exit 1
grep -E '^\{' gpurun_out/r3s2a/bench_default.log | cut -c1-300
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3s2a/prof -o st -- \
  python3 bench.py --steps 20 --warmup 3 > gpurun_out/r3s2a/bench_traced.log 2>&1 || exit 1
f=$(find gpurun_out/r3s2a/prof -name "*kernel_trace.csv" | head -n 1)
python scripts/step_breakdown.py "$f" --steps 15 --top 60 --gaps 6 --dump-step gpurun_out/r3s2a/one_step.txt > gpurun_out/r3s2a/breakdown.txt && head -30 gpurun_out/r3s2a/breakdown.txt
rm -f "$f"
