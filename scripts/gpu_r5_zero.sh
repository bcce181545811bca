# ZeRO-1 deferred all-gather on the GPU: the RCCL tests (one-rank schedule + in-place gather), then a two-rank
# rehearsal on the one GPU (gloo over CUDA tensors, IIT_REHEARSE_ONE_GPU=1) with the gather deferred to the next
# forward's per-block gates vs waited right after Adam -- same weight checksum, step time of each; then the
# eval_information timing (probe sweep on the activation bank vs the reference engine).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5z
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_dp_rccl_gpu.py \
  > gpurun_out/r5z/rccl_tests.log 2>&1 || { echo "rccl tests failed"; tail -30 gpurun_out/r5z/rccl_tests.log; exit 1; }
tail -3 gpurun_out/r5z/rccl_tests.log
for ov in 1 0; do
  IIT_REHEARSE_ONE_GPU=1 IIT_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2971$ov scripts/bench_families.py \
    --family llama-tiny-causal --zero 1 --zero-overlap $ov --steps 20 --warmup 3 > gpurun_out/r5z/zero_ov$ov.log 2>&1 \
    || { echo "rehearsal ov=$ov failed"; tail -30 gpurun_out/r5z/zero_ov$ov.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"weight_checksum": [-0-9.e]*\|"zero_overlap_gather": [a-z]*' gpurun_out/r5z/zero_ov$ov.log
done
timeout -k 10 800 python -u scripts/eval_pvr_r4.py --skip-causality > gpurun_out/r5z/info.log 2>&1 \
  || { echo "info failed"; tail -30 gpurun_out/r5z/info.log; exit 1; }
grep "\[pvr\]" gpurun_out/r5z/info.log
# Llama-3-8B S=512 kernel breakdown at HEAD (hook_z spliced in the flash-attention store: no splice_kernel rows)
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5z/llprof -o ll -- python3 scripts/bench_families.py \
  --family llama3-8b-causal --seq 512 --steps 3 --warmup 2 > gpurun_out/r5z/llama_prof.log 2>&1 \
  || { echo "llama trace failed"; tail -20 gpurun_out/r5z/llama_prof.log; exit 1; }
grep -E '^\{' gpurun_out/r5z/llama_prof.log | cut -c1-200
f=$(find gpurun_out/r5z/llprof -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 3 --per-step-adam 3 --top 45 > gpurun_out/r5z/llama_breakdown.txt \
  && head -12 gpurun_out/r5z/llama_breakdown.txt; grep -c splice_kernel gpurun_out/r5z/llama_breakdown.txt || true; rm -f "$f"
