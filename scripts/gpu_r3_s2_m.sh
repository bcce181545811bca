# Round 3 session 2: LN backward reading the bf16 xhat (LNPre) -> tests, bench A/B (IIT_LN_XHAT16 on / off).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3s2m
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_hip_kernels.py tests/test_hip_model.py tests/test_paired.py tests/test_graphs.py tests/test_fused_norm.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|FAIL|assert" $O/tests.log | head -30; exit $rc; }
for i in 1 2; do
timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > $O/bench_$i.log 2>&1 || { tail -30 $O/bench_$i.log; exit 1; }
grep -E '^\{' $O/bench_$i.log | cut -c1-200
IIT_LN_XHAT16=0 timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > $O/bench_off_$i.log 2>&1 || { tail -30 $O/bench_off_$i.log; exit 1; }
grep -E '^\{' $O/bench_off_$i.log | cut -c1-200
done
