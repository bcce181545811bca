# eval_information timing split (activation bank vs per-batch captures vs the reference engine), and the run-to-run
# spread of the ZeRO-1 rehearsal's weight checksum with the gather waited right after Adam (no deferral).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5i
IIT_PROBE_TIMING=1 timeout -k 10 700 python -u scripts/eval_pvr_r4.py --skip-causality --epochs 2 --train-size 20000 \
  --info-engines native native_nobank reference > gpurun_out/r5i/info.log 2>&1 \
  || { echo "info failed"; tail -30 gpurun_out/r5i/info.log; exit 1; }
grep "\[pvr\]\|\[probe timing\]" gpurun_out/r5i/info.log
for rep in a b; do
  IIT_REHEARSE_ONE_GPU=1 IIT_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2972$([ $rep = a ] && echo 1 || echo 2) scripts/bench_families.py \
    --family llama-tiny-causal --zero 1 --zero-overlap 0 --steps 20 --warmup 3 > gpurun_out/r5i/zero_$rep.log 2>&1 \
    || { echo "rehearsal $rep failed"; tail -30 gpurun_out/r5i/zero_$rep.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"weight_checksum": [-0-9.e]*' gpurun_out/r5i/zero_$rep.log
done
