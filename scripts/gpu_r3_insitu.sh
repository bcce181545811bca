# Round 3: in-context GEMM selection (scripts/tune_gemm_in_situ.py), then the bench with that table.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
IIT_GEMM_TABLE=0 timeout -k 10 900 python3 -u scripts/tune_gemm_in_situ.py --out gpurun_out/gemm_decisions_in_situ.json \
  > gpurun_out/tune_in_situ.log 2>&1 || { echo tune failed; tail -30 gpurun_out/tune_in_situ.log; exit 1; }
tail -3 gpurun_out/tune_in_situ.log
cp gpurun_out/gemm_decisions_in_situ.json iit_amd/ops/tuned/gemm_decisions_gfx950.json
timeout -k 10 300 python3 -u bench.py > gpurun_out/bench_insitu.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_insitu.log; exit 1; }
tail -1 gpurun_out/bench_insitu.log
