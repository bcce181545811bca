# Round 3 session 2: batch copied into the static graph inputs with one multi-tensor launch -> graph tests, bench A/B.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3s2o
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_graphs.py tests/test_hip_model.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|FAIL|assert" $O/tests.log | head -30; exit $rc; }
for i in 1 2; do
timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > $O/bench_on_$i.log 2>&1 || { tail -30 $O/bench_on_$i.log; exit 1; }
echo "foreach copy: $(grep -E '^\{' $O/bench_on_$i.log | cut -c100-200)"
IIT_FOREACH_COPY=0 timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > $O/bench_off_$i.log 2>&1 || { tail -30 $O/bench_off_$i.log; exit 1; }
echo "copy per tensor: $(grep -E '^\{' $O/bench_off_$i.log | cut -c100-200)"
done
