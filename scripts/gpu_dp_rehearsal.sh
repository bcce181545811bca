# Multi-rank data-parallel rehearsal on a one-GPU box: 2 ranks share cuda:0 over gloo (RCCL refuses two ranks on
# one device) and run the headline bench end to end -- rank-sharded batches, broadcast of the arena, staged
# backward graphs with eager range all-reduces between replays, max-over-ranks timing.  Not a measurement.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export IIT_REHEARSE_ONE_GPU=1 IIT_DIST_BACKEND=gloo
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 4 --warmup 3 > gpurun_out/dp_rehearsal.log 2>&1
rc=$?
tail -5 gpurun_out/dp_rehearsal.log
exit $rc
