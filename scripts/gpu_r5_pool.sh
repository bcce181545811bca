# NHWC byte-argmax max pool (ops/bn.py MaxPool3s2Fn): PVR GPU tests, bf16 step A/B
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5pool; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bn_fused.py tests/test_mnist_pvr_gpu.py > $O/t.log 2>&1 \
  || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for fp in 0 1 0 1; do
  IIT_FUSED_POOL=$fp timeout -k 10 300 python3 -u scripts/bench_families.py --family pvr-resnet18 --dtype bf16 --steps 20 --warmup 3 > $O/pvr$fp.log 2>&1 || { tail -20 $O/pvr$fp.log; exit 1; }
  echo "pool=$fp $(grep -o '"ms_per_step": [0-9.]*\|"val_IIA": [0-9.]*' $O/pvr$fp.log | tr '\n' ' ')"
done
