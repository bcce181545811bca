# eval_information timing after an untimed warm-up of every engine; ZeRO-1 rehearsal with poisoned foreign pieces
# (IIT_ZERO_POISON=1: NaN until a gate finishes the bucket) and the deferred gather, twice (run-to-run spread).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5j
for rep in 1 2; do
  IIT_ZERO_POISON=1 IIT_REHEARSE_ONE_GPU=1 IIT_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2973$rep scripts/bench_families.py \
    --family llama-tiny-causal --zero 1 --zero-overlap 1 --steps 20 --warmup 3 > gpurun_out/r5j/zero_$rep.log 2>&1 \
    || { echo "rehearsal $rep failed"; tail -30 gpurun_out/r5j/zero_$rep.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"weight_checksum": [-0-9.e]*\|"last_train_losses": {[^}]*}\|"optimizer_skipped_steps": [0-9]*' gpurun_out/r5j/zero_$rep.log
done
IIT_PROBE_TIMING=1 timeout -k 10 700 python -u scripts/eval_pvr_r4.py --skip-causality --epochs 2 --train-size 20000 \
  --info-engines native native_nobank reference > gpurun_out/r5j/info.log 2>&1 \
  || { echo "info failed"; tail -30 gpurun_out/r5j/info.log; exit 1; }
grep "\[pvr\]\|\[probe timing\]" gpurun_out/r5j/info.log
