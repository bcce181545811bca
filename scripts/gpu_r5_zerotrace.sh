# ZeRO-1 deferred all-gather on the one-GPU 2-rank rehearsal (gloo over CUDA tensors): rank 0 traced with
# --kernel-trace --memory-copy-trace (no counters), the gather deferred (overlap=1) vs waited right after Adam (0)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5zt; mkdir -p $O
for ov in 1 0; do
  export MASTER_ADDR=127.0.0.1 MASTER_PORT=2976$ov WORLD_SIZE=2 IIT_REHEARSE_ONE_GPU=1 IIT_DIST_BACKEND=gloo
  RANK=1 LOCAL_RANK=1 timeout -k 10 300 python3 scripts/bench_families.py --family llama-tiny-causal --zero 1 --zero-overlap $ov --steps 20 --warmup 3 > $O/r1_ov$ov.log 2>&1 &
  pid=$!
  RANK=0 LOCAL_RANK=0 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/ov$ov -o r0 -- python3 scripts/bench_families.py --family llama-tiny-causal --zero 1 --zero-overlap $ov --steps 20 --warmup 3 > $O/r0_ov$ov.log 2>&1
  rc=$?
  wait $pid; rc1=$?
  [ $rc -eq 0 ] && [ $rc1 -eq 0 ] || { echo "ov=$ov failed rc=$rc rc1=$rc1"; tail -20 $O/r0_ov$ov.log; tail -20 $O/r1_ov$ov.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"weight_checksum": [-0-9.e]*' $O/r0_ov$ov.log | tr '\n' ' '; echo
  python3 scripts/zero_overlap_trace.py $O/ov$ov
done
