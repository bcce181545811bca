# Round 3 session 2: fused gradient norm (weight-gradient GEMMs add the sums of squares; the norm pass skips them)
# -> kernel / model / norm tests, bench A/B (IIT_FUSED_NORM on / off), kernel trace.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3s2g
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_fused_norm.py tests/test_gemm_dual.py tests/test_hip_kernels.py tests/test_hip_model.py tests/test_graphs.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|FAIL|assert" $O/tests.log | head -30; exit $rc; }
timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep -E '^\{' $O/bench.log | cut -c1-200
IIT_FUSED_NORM=0 timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > $O/bench_nonorm.log 2>&1 || { tail -30 $O/bench_nonorm.log; exit 1; }
grep -E '^\{' $O/bench_nonorm.log | cut -c1-200
timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > $O/bench2.log 2>&1 || { tail -30 $O/bench2.log; exit 1; }
grep -E '^\{' $O/bench2.log | cut -c1-200
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o st -- \
  python3 bench.py --steps 20 --warmup 3 > $O/bench_traced.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_trace.csv" | head -n 1)
python scripts/step_breakdown.py "$f" --steps 15 --top 70 --gaps 6 --dump-step $O/one_step.txt > $O/breakdown.txt && head -45 $O/breakdown.txt
rm -f "$f"
timeout -k 10 400 python3 -u scripts/bench_adam.py > $O/adam.log 2>&1 || { tail -20 $O/adam.log; exit 1; }
cat $O/adam.log
