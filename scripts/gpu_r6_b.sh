# round 6, call B: the chunk-partial BatchNorm (tests + PVR bf16 / fp32 steps + a kernel trace of the bf16 step), then the
# headline-shape GEMM microbench (dispatch choice vs the 256 x 256 four-wave tile vs hipBLASLt)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6b; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_bn_fused.py tests/test_mnist_pvr_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_bn.log 2>&1
rc=$?; tail -3 $O/pytest_bn.log; [ $rc -eq 0 ] || { tail -40 $O/pytest_bn.log; exit $rc; }
for dt in bf16 fp32; do
  timeout -k 10 300 python3 scripts/bench_families.py --family pvr-resnet18 --dtype $dt --steps 20 --warmup 3 > $O/pvr_$dt.log 2>&1 || { tail -20 $O/pvr_$dt.log; exit 2; }
  grep -E '^\{' $O/pvr_$dt.log | cut -c1-260
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o pv -- python3 scripts/bench_families.py --family pvr-resnet18 --dtype bf16 --steps 10 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 3; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 6 --top 45 --gaps 5 > $O/pvr_breakdown.txt && head -30 $O/pvr_breakdown.txt | cut -c1-160; rm -rf $O/prof
timeout -k 10 500 python3 scripts/bench_headline_gemms.py --rounds 3 > $O/headline_gemms.log 2>&1 || { tail -20 $O/headline_gemms.log; exit 4; }
cat $O/headline_gemms.log | grep -v amdgpu.ids | cut -c1-300
