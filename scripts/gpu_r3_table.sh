# Round 3: re-autotune every GEMM shape of the headline step (new 2/3/4-workgroup-per-CU tiles), export the
# decision table, then bench with it and profile one short run.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
IIT_GEMM_TABLE=0 IIT_GEMM_TABLE_EXPORT=gpurun_out/gemm_decisions_gfx950.json IIT_GEMM_REPORT=gpurun_out/gemm_report.txt \
  timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 3 > gpurun_out/bench_tune.log 2>&1 || { echo tune failed; tail -20 gpurun_out/bench_tune.log; exit 1; }
tail -1 gpurun_out/bench_tune.log
cp gpurun_out/gemm_decisions_gfx950.json iit_amd/ops/tuned/gemm_decisions_gfx950.json
timeout -k 10 300 python3 -u bench.py > gpurun_out/bench_r3.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_r3.log; exit 1; }
tail -1 gpurun_out/bench_r3.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 20 --warmup 3 > gpurun_out/prof/bench_stdout.log 2>&1
echo "rocprof rc=$?"
find gpurun_out/prof -name "*kernel_trace.csv" | head -2
