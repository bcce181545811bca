# fused NHWC BatchNorm for fp32 activations: tests, PVR fp32 step NCHW (module path) vs channels-last (fused)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5bf; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bn_fused.py tests/test_mnist_pvr_gpu.py > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for cl in 0 1 0 1; do
  timeout -k 10 300 python3 -u scripts/bench_families.py --family pvr-resnet18 --dtype fp32 --channels-last $cl --steps 20 --warmup 3 > $O/cl$cl.log 2>&1 || { tail -20 $O/cl$cl.log; exit 1; }
  echo "cl=$cl $(grep -o '"ms_per_step": [0-9.]*\|"val_IIA": [0-9.]*' $O/cl$cl.log | tr '\n' ' ')"
done
