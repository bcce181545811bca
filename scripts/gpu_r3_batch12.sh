# Round 3 batch 12: paired tests (incl. staged cuts), the DP schedule on one GPU (1-rank RCCL, forced reducer:
# staged backward graphs + range all-reduces, now with the paired forward), 2-rank gloo rehearsal, step profile.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3n
run() {
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/r3n/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; grep -v amdgpu.ids "gpurun_out/r3n/$name.log" | grep -vE '^[EW]2026' | tail -3 | cut -c1-400
  if [ $rc -ge 124 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
  return 0
}
run tests 400 python3 -u -m pytest tests/test_paired.py tests/test_dp_rccl_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread
IIT_DP_FORCE_REDUCER=1 run dp1_rccl 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 30 --warmup 5
IIT_DP_FORCE_REDUCER=1 IIT_PAIRED=0 run dp1_rccl_unpaired 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 1 --steps 30 --warmup 5
IIT_REHEARSE_ONE_GPU=1 IIT_DIST_BACKEND=gloo run dp2_gloo 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 4 --warmup 3
echo "batch done"
