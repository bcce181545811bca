# fp32 PVR: fused NHWC BN + pool (fp32 instantiations); tests; step A/B; train.py short run (channels-last default)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5bf2; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bn_fused.py tests/test_mnist_pvr_gpu.py > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for cl in 0 1 0 1; do
  timeout -k 10 300 python3 -u scripts/bench_families.py --family pvr-resnet18 --dtype fp32 --channels-last $cl --steps 20 --warmup 3 > $O/cl$cl.log 2>&1 || { tail -20 $O/cl$cl.log; exit 1; }
  echo "fp32 cl=$cl $(grep -o '"ms_per_step": [0-9.]*\|"val_IIA": [0-9.]*' $O/cl$cl.log | tr '\n' ' ')"
done
timeout -k 10 300 python3 -u scripts/bench_families.py --family pvr-resnet18 --dtype bf16 --steps 20 --warmup 3 > $O/bf16.log 2>&1 || { tail -20 $O/bf16.log; exit 1; }
echo "bf16 $(grep -o '"ms_per_step": [0-9.]*\|"val_IIA": [0-9.]*' $O/bf16.log | tr '\n' ' ')"
timeout -k 10 400 python3 -u train.py --train-size 20000 --test-size 2000 --epochs 2 > $O/train.log 2>&1 || { tail -20 $O/train.log; exit 1; }
grep -E "val/IIA|val/accuracy|epoch|done" $O/train.log | tail -6
