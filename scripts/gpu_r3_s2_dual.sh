# Round 3 session 2: dual dX+dW GEMM launch -> kernel tests, bench A/B (dual on / off), model tests, step trace.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3s2b
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gemm_dual.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests_dual.log 2>&1
rc=$?; tail -3 $O/tests_dual.log; [ $rc -eq 0 ] || { tail -40 $O/tests_dual.log; exit $rc; }
IIT_GEMM_REPORT=$O/gemm_report_dual.txt IIT_GEMM_TABLE_EXPORT=$O/table_dual.json timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > $O/bench_dual.log 2>&1 || { tail -30 $O/bench_dual.log; exit 1; }
grep -E '^\{' $O/bench_dual.log | cut -c1-220
IIT_GEMM_DUAL=0 timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > $O/bench_nodual.log 2>&1 || { tail -30 $O/bench_nodual.log; exit 1; }
grep -E '^\{' $O/bench_nodual.log | cut -c1-220
grep "^pair" $O/gemm_report_dual.txt | cut -c1-250
timeout -k 10 600 python3 -u -m pytest tests/test_hip_model.py tests/test_paired.py tests/test_graphs.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests_model.log 2>&1
rc=$?; tail -3 $O/tests_model.log; [ $rc -eq 0 ] || { tail -40 $O/tests_model.log; exit $rc; }
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o st -- \
  python3 bench.py --steps 20 --warmup 3 > $O/bench_traced.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_trace.csv" | head -n 1)
python scripts/step_breakdown.py "$f" --steps 15 --top 60 --gaps 6 --dump-step $O/one_step.txt > $O/breakdown.txt && head -40 $O/breakdown.txt
rm -f "$f"
