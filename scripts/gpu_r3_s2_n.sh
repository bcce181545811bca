# Round 3 session 2: in-context re-tune with the residual reduction splits always competing -> tests, tune,
# benches (new table x2, shipped table).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3s2n
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_hip_kernels.py tests/test_hip_model.py tests/test_paired.py tests/test_graphs.py tests/test_fused_norm.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|FAIL|assert" $O/tests.log | head -30; exit $rc; }
IIT_GEMM_TABLE=0 timeout -k 10 700 python3 -u scripts/tune_gemm_in_situ.py --out $O/table_insitu.json \
  --report $O/insitu_report.txt > $O/tune.log 2>&1 || { echo tune failed; tail -30 $O/tune.log; exit 1; }
tail -1 $O/tune.log
for i in 1 2; do
IIT_GEMM_TABLE=$O/table_insitu.json timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > $O/bench_new_$i.log 2>&1 || { tail -30 $O/bench_new_$i.log; exit 1; }
echo "new table: $(grep -E '^\{' $O/bench_new_$i.log | cut -c100-200)"
timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > $O/bench_shipped_$i.log 2>&1 || { tail -30 $O/bench_shipped_$i.log; exit 1; }
echo "shipped table: $(grep -E '^\{' $O/bench_shipped_$i.log | cut -c100-200)"
done
grep -v dual $O/insitu_report.txt | grep ", 2, 2," | cut -c1-250
