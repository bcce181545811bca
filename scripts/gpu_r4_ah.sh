# Round 4 (session 2): ragged-split tails (the 81-column / 81-step remainders of the vocabulary GEMMs) on the repo's
# kernels.  GEMM tests, then A/B x3 against IIT_GEMM_TAIL_LIBRARY=1 (hipBLASLt allowed on the tails), then a kernel
# trace of the default configuration (expect zero Cijk rows).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4ah
mkdir -p $O
j() { grep -E '^\{' $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "pairs/s", d["ms_per_step"], "ms")'; }
timeout -k 10 400 python3 -u -m pytest tests/test_gemm_glds.py tests/test_gemm_dispatch.py tests/test_headline_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in a b c; do
  IIT_GEMM_REPORT=$O/decisions_new_$r.txt timeout -k 10 300 python3 -u bench.py > $O/bench_new_$r.log 2>&1 || { tail -30 $O/bench_new_$r.log; exit 1; }
  echo "tails on own kernels $r: $(j bench_new_$r)"
  IIT_GEMM_TAIL_LIBRARY=1 timeout -k 10 300 python3 -u bench.py > $O/bench_lib_$r.log 2>&1 || { tail -30 $O/bench_lib_$r.log; exit 1; }
  echo "tails may use hipBLASLt $r: $(j bench_lib_$r)"
done
grep -E "N=    81|K=    81" $O/decisions_new_a.txt | cut -c1-160
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o b -- python3 bench.py --steps 20 --warmup 3 > $O/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/prof.log; exit $rc; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -n 1)
python3 scripts/step_breakdown.py "$f" --steps 15 --top 120 --gaps 5 --dump-step $O/step_seq.txt > $O/step_breakdown.txt && head -3 $O/step_breakdown.txt
echo "Cijk rows: $(grep -c Cijk $O/step_breakdown.txt || true)"
rm -rf $O/prof
