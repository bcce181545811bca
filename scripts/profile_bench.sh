# rocprofv3 kernel trace + stats of a short bench run; summaries copied to profiles/ by the caller
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 5 --warmup 2 "$@" > gpurun_out/prof/bench_stdout.log 2>&1
rc=$?
echo "rocprof rc=$rc"
tail -3 gpurun_out/prof/bench_stdout.log
find gpurun_out/prof -name "*stats*" | head
