# Round 3 session 2: in-context re-tune with the residual reduction splits always competing -> table, bench new vs shipped.
# (8-wave and deep-ring dual families always compete), bench with the new table vs the shipped one, BERT family.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3s2l
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_hip_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|FAIL|assert" $O/tests.log | head -30; exit $rc; }
IIT_GEMM_TABLE=0 timeout -k 10 700 python3 -u scripts/tune_gemm_in_situ.py --out $O/table_insitu.json \
  --report $O/insitu_report.txt > $O/tune.log 2>&1 || { echo tune failed; tail -30 $O/tune.log; exit 1; }
tail -2 $O/tune.log
IIT_GEMM_TABLE=$O/table_insitu.json IIT_GEMM_REPORT=$O/report_insitu.txt timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > $O/bench_insitu.log 2>&1 || { tail -30 $O/bench_insitu.log; exit 1; }
grep -E '^\{' $O/bench_insitu.log | cut -c1-200
timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > $O/bench_shipped.log 2>&1 || { tail -30 $O/bench_shipped.log; exit 1; }
grep -E '^\{' $O/bench_shipped.log | cut -c1-200
IIT_GEMM_TABLE=$O/table_insitu.json timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > $O/bench_insitu2.log 2>&1 || { tail -30 $O/bench_insitu2.log; exit 1; }
grep -E '^\{' $O/bench_insitu2.log | cut -c1-200
grep dual $O/insitu_report.txt | cut -c1-330
