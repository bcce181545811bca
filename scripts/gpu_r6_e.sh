# round 6, call E: BN (atomic default, two-level in deterministic mode) + conv tests, the PVR bf16 step with the
# implicit-GEMM convolutions (untraced + kernel trace), the conv decisions, and the headline bench
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6e; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_bn_fused.py tests/test_conv_nhwc.py tests/test_mnist_pvr_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert |FAILED" $O/pytest.log | head -30; tail -30 $O/pytest.log; exit $rc; }
for cv in auto 0; do
  IIT_CONV_HIP=$cv timeout -k 10 300 python3 scripts/bench_families.py --family pvr-resnet18 --dtype bf16 --steps 30 --warmup 3 > $O/pvr_conv_$cv.log 2>&1 || { tail -20 $O/pvr_conv_$cv.log; exit 2; }
  echo "pvr conv=$cv: $(grep -E '^\{' $O/pvr_conv_$cv.log | cut -c150-230)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o pv -- python3 scripts/bench_families.py --family pvr-resnet18 --dtype bf16 --steps 10 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 3; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 6 --top 50 --gaps 5 > $O/pvr_breakdown.txt && head -12 $O/pvr_breakdown.txt | cut -c1-160; rm -rf $O/prof
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 4; }
grep -E '^\{' $O/bench.log | cut -c1-260
