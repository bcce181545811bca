# ZeRO-1 rehearsal (2 ranks on one GPU, gloo) with IIT_ZERO_POISON=1: foreign pieces NaN and each bucket's gather issued only
# when a gate finishes it -- a weight read that bypasses the gates always reads NaN.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5k
for rep in 1 2; do
  IIT_ZERO_POISON=1 IIT_REHEARSE_ONE_GPU=1 IIT_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2974$rep scripts/bench_families.py \
    --family llama-tiny-causal --zero 1 --zero-overlap 1 --steps 20 --warmup 3 > gpurun_out/r5k/zero_$rep.log 2>&1 \
    || { echo "rehearsal $rep failed"; tail -30 gpurun_out/r5k/zero_$rep.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"weight_checksum": [-0-9.e]*\|"last_train_losses": {[^}]*}\|"optimizer_skipped_steps": [0-9]*' gpurun_out/r5k/zero_$rep.log
done
