# Round 3 session 2: a phase's Adam overlapped with the next phase's forward (per-stage chunks on a side stream)
# -> overlap tests, graph / model tests, bench A/B (IIT_ADAM_OVERLAP=0), kernel trace of the headline step.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3s2q
mkdir -p $O
IIT_TEST_ADAM_OVERLAP=1 timeout -k 10 600 python3 -u -m pytest tests/test_adam_overlap.py tests/test_graphs.py tests/test_hip_model.py tests/test_fused_norm.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|FAIL|assert" $O/tests.log | head -30; exit $rc; }
for i in 1 2; do
IIT_ADAM_OVERLAP=1 timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > $O/bench_on_$i.log 2>&1 || { tail -30 $O/bench_on_$i.log; exit 1; }
echo "overlapped Adam: $(grep -E '^\{' $O/bench_on_$i.log | cut -c100-200)"
IIT_ADAM_OVERLAP=0 timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > $O/bench_off_$i.log 2>&1 || { tail -30 $O/bench_off_$i.log; exit 1; }
echo "serial Adam: $(grep -E '^\{' $O/bench_off_$i.log | cut -c100-200)"
done
IIT_ADAM_OVERLAP=1 timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o st -- \
  python3 bench.py --steps 20 --warmup 3 > $O/bench_traced.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_trace.csv" | head -n 1)
python scripts/step_breakdown.py "$f" --steps 15 --top 40 --gaps 6 --dump-step $O/one_step.txt > $O/breakdown.txt && head -30 $O/breakdown.txt
rm -f "$f"
