# Round 4 (session 2): gradient-arena memset with 128 ranges per launch (was 64): the zero_ranges GPU test, the
# launch count in the headline step (expect 2 per phase, was 3), bench x2
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4ak
mkdir -p $O
j() { grep -E '^\{' $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "pairs/s", d["ms_per_step"], "ms")'; }
timeout -k 10 300 python3 -u -m pytest tests/test_hip_kernels.py tests/test_headline_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_a.log 2>&1 || { tail -30 $O/bench_a.log; exit 1; }
echo "bench a: $(j bench_a)"
timeout -k 10 300 python3 -u bench.py > $O/bench_b.log 2>&1 || { tail -30 $O/bench_b.log; exit 1; }
echo "bench b: $(j bench_b)"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o b -- python3 bench.py --steps 20 --warmup 3 > $O/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/prof.log; exit $rc; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -n 1)
python3 scripts/step_breakdown.py "$f" --steps 15 --top 120 --gaps 5 > $O/step_breakdown.txt && head -3 $O/step_breakdown.txt
grep -E "zero_ranges|Cijk" $O/step_breakdown.txt | cut -c1-100
rm -rf $O/prof
