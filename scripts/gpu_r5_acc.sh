# fused fp32 += bf16 gradient accumulate (torch_ops._accumulate): tests + PVR bf16 step
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5acc; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bn_fused.py tests/test_mnist_pvr_gpu.py tests/test_llama_ops.py tests/test_hip_model.py > $O/t.log 2>&1 \
  || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in a b; do
  timeout -k 10 300 python3 -u scripts/bench_families.py --family pvr-resnet18 --dtype bf16 --steps 20 --warmup 3 > $O/pvr$r.log 2>&1 || { tail -20 $O/pvr$r.log; exit 1; }
  echo "run $r $(grep -o '"ms_per_step": [0-9.]*\|"val_IIA": [0-9.]*' $O/pvr$r.log | tr '\n' ' ')"
done
