# The full training loop (BaseModelPair.train: graphed phases, staged DP backward, epoch metric all-reduce, per-epoch
# HIP-event throughput) with 2 data-parallel ranks sharing one GPU over gloo -- the multi-rank train() path end to end
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export IIT_REHEARSE_ONE_GPU=1 IIT_DIST_BACKEND=gloo IIT_PROFILE=1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29541 scripts/time_to_iia.py --model gpt2-small --dtype bf16 --epochs 3 --num-samples 3000 \
  > gpurun_out/dp_train_rehearsal.log 2>&1
rc=$?
grep -E "Epoch|\[perf\]|metric" gpurun_out/dp_train_rehearsal.log | cut -c1-260
exit $rc
