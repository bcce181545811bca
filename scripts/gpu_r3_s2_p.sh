# Round 3 session 2: one gsq atomic per workgroup, no fused bias sums on the vocabulary-wide unembed gradient
# -> fused-sum tests, bench A/B against the old vocab-wide fusion, kernel trace of the headline step.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3s2p
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gemm_dual.py tests/test_fused_norm.py tests/test_hip_kernels.py tests/test_hip_model.py tests/test_graphs.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|FAIL|assert" $O/tests.log | head -30; exit $rc; }
for i in 1 2; do
timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > $O/bench_new_$i.log 2>&1 || { tail -30 $O/bench_new_$i.log; exit 1; }
echo "layer biases fused: $(grep -E '^\{' $O/bench_new_$i.log | cut -c100-200)"
IIT_FUSED_BIAS_MAX_N=1000000 timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > $O/bench_old_$i.log 2>&1 || { tail -30 $O/bench_old_$i.log; exit 1; }
echo "vocab bias fused too: $(grep -E '^\{' $O/bench_old_$i.log | cut -c100-200)"
done
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o st -- \
  python3 bench.py --steps 20 --warmup 3 > $O/bench_traced.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_trace.csv" | head -n 1)
python scripts/step_breakdown.py "$f" --steps 15 --top 70 --gaps 6 --dump-step $O/one_step.txt > $O/breakdown.txt && head -30 $O/breakdown.txt
rm -f "$f"
