# round 6, call A: GPU tests + smoke + driver bench at HEAD, then the multi-rank launch path rehearsed on ONE GPU:
# bench.py --gpus 2 with no launcher (self-launch), two gloo ranks sharing the card (IIT_REHEARSE_ONE_GPU), weak and
# strong scaling (the driver's 8-GPU node uses RCCL, one rank per GPU)
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_final.sh || exit $?
mkdir -p gpurun_out/r6a
IIT_REHEARSE_ONE_GPU=1 IIT_DIST_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --steps 5 --warmup 2 \
  > gpurun_out/r6a/selflaunch_weak.log 2>&1 || { echo "self-launch weak failed"; tail -30 gpurun_out/r6a/selflaunch_weak.log; exit 5; }
grep -E '^\{' gpurun_out/r6a/selflaunch_weak.log | cut -c1-400
IIT_REHEARSE_ONE_GPU=1 IIT_DIST_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --steps 5 --warmup 2 --global-batch 256 \
  > gpurun_out/r6a/selflaunch_strong.log 2>&1 || { echo "self-launch strong failed"; tail -30 gpurun_out/r6a/selflaunch_strong.log; exit 6; }
grep -E '^\{' gpurun_out/r6a/selflaunch_strong.log | cut -c1-400
