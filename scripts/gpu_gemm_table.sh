# Measure the GEMM decisions with the table off (fresh autotuning) for the headline model and export them as the
# shipped table; then the bf16 time-to-IIA run reads it (no autotuning of known shapes in epoch 0)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tti
IIT_GEMM_TABLE=0 IIT_GEMM_TABLE_EXPORT=gpurun_out/gemm_decisions_gfx950.json timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_export.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_export.log; exit 3; }
tail -1 gpurun_out/bench_export.log | cut -c1-200
cp gpurun_out/gemm_decisions_gfx950.json iit_amd/ops/tuned/gemm_decisions_gfx950.json
timeout -k 10 400 python -u scripts/time_to_iia.py --model gpt2-small --dtype bf16 --epochs 61 > gpurun_out/tti/gpt2_bf16_61_table.log 2>&1
rc=$?; tail -1 gpurun_out/tti/gpt2_bf16_61_table.log | cut -c1-500; exit $rc
