# Profile + reference-equivalent measurement (run after scripts/gpu_check.sh in the same gpurun call).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 40 --warmup 3 > gpurun_out/bench_prof.log 2>&1 || { echo prof failed $?; tail -20 gpurun_out/bench_prof.log; exit 5; }
f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -n 1)
n=$(sed -n 's/.*train steps executed in this process: \([0-9]*\).*/\1/p' gpurun_out/bench_prof.log)
python scripts/summarize_profile.py "$f" "$n" 45 > gpurun_out/kernel_stats_top.txt && head -30 gpurun_out/kernel_stats_top.txt
if [ "${IIT_REF_BENCH:-1}" = "1" ]; then
  timeout -k 10 400 python bench.py --engine reference --dtype fp32 --graphs 0 --steps 5 --warmup 2 > gpurun_out/bench_reference.log 2>&1 || { echo ref bench failed $?; tail -20 gpurun_out/bench_reference.log; exit 6; }
  tail -1 gpurun_out/bench_reference.log
fi
