# Round 3 batch 6: in-context GEMM table with the paired forward (M = 2T source+base GEMMs), bench, full GPU suite.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3g
IIT_GEMM_TABLE=0 timeout -k 10 900 python3 -u scripts/tune_gemm_in_situ.py --out gpurun_out/r3g/gemm_decisions_in_situ.json \
  --report gpurun_out/r3g/gemm_in_situ_report.txt > gpurun_out/r3g/tune_in_situ.log 2>&1 || { echo tune failed; tail -30 gpurun_out/r3g/tune_in_situ.log; exit 1; }
tail -3 gpurun_out/r3g/tune_in_situ.log
cp gpurun_out/r3g/gemm_decisions_in_situ.json iit_amd/ops/tuned/gemm_decisions_gfx950.json
timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > gpurun_out/r3g/bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/r3g/bench.log; exit 1; }
grep -E '^\{' gpurun_out/r3g/bench.log | cut -c1-250
timeout -k 10 300 python3 -u bench.py > gpurun_out/r3g/bench_default.log 2>&1 || { echo bench failed; exit 1; }
grep -E '^\{' gpurun_out/r3g/bench_default.log | cut -c1-250
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3g/gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r3g/gpu_tests.log; echo "tests rc=$rc"
