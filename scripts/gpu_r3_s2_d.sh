# Round 3 session 2: fused bias sums (weight-gradient GEMM colsum of dY) + wave-parallel IOI HL label -> kernel and
# model tests, bench A/B (fused bias sums on / off).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3s2d
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gemm_dual.py tests/test_ioi_hl_kernel.py tests/test_hip_model.py tests/test_paired.py tests/test_graphs.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|error|FAIL|assert" $O/tests.log | head -30; exit $rc; }
IIT_GEMM_REPORT=$O/gemm_report.txt timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep -E '^\{' $O/bench.log | cut -c1-200
IIT_FUSED_BIAS_SUMS=0 timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > $O/bench_nofuse.log 2>&1 || { tail -30 $O/bench_nofuse.log; exit 1; }
grep -E '^\{' $O/bench_nofuse.log | cut -c1-200
timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > $O/bench2.log 2>&1 || { tail -30 $O/bench2.log; exit 1; }
grep -E '^\{' $O/bench2.log | cut -c1-200
