# Rehearse the multi-GPU data-parallel path on ONE GPU: a one-rank RCCL process group with the reducer forced
# on, so bench.py runs exactly the DP schedule (staged backward graphs, range all-reduces over RCCL between
# replays, row-sparse embedding reduction, averaged gradients) -- everything but more than one rank.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
IIT_DP_FORCE_REDUCER=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/dp_rehearsal.log 2>&1
rc=$?
echo "rehearsal rc=$rc"
grep -v "amdgpu.ids" gpurun_out/dp_rehearsal.log | tail -5
exit $rc
