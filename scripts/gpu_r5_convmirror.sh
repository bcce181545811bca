# ResNet convs on the arena's bf16 mirror under autocast (resnet.Conv2d): PVR tests, bf16 step A/B
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5cm; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bn_fused.py tests/test_mnist_pvr_gpu.py > $O/t.log 2>&1 \
  || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for cm in 0 1 0 1; do
  IIT_CONV_MIRROR=$cm timeout -k 10 300 python3 -u scripts/bench_families.py --family pvr-resnet18 --dtype bf16 --steps 20 --warmup 3 > $O/pvr$cm.log 2>&1 || { tail -20 $O/pvr$cm.log; exit 1; }
  echo "mirror=$cm $(grep -o '"ms_per_step": [0-9.]*\|"val_IIA": [0-9.]*' $O/pvr$cm.log | tr '\n' ' ')"
done
