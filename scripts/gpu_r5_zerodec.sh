# is the deferred-gather checksum difference a GEMM-autotune decision difference?  GEMM decision reports per run.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5zd; mkdir -p $O
for tag in d1 n1 d2 n2; do
  ov=$([ ${tag:0:1} = d ] && echo 1 || echo 0)
  IIT_GEMM_REPORT=$O/gemm_$tag.txt IIT_REHEARSE_ONE_GPU=1 IIT_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 297${tag:1:1}$ov scripts/bench_families.py \
    --family llama-tiny-causal --zero 1 --zero-overlap $ov --steps 20 --warmup 3 > $O/$tag.log 2>&1 \
    || { echo "$tag failed"; tail -30 $O/$tag.log; exit 1; }
  echo "$tag $(grep -o '"weight_checksum": [-0-9.e]*' $O/$tag.log)"
done
for f in $O/gemm_*.txt; do echo "$f $(md5sum < $f | cut -c1-8) $(wc -l < $f)"; done
