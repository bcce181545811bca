# Round 4 (session 2): the last library GEMM in the headline step is the 81-column tail of the ragged unembed
# weight gradient (768 x 81 x 256, mode 3, fp32 store).  A/B x3: shipped table vs the same table with hipBLASLt
# excluded at that key (the hand-written candidates decide it), then a kernel trace of the excluded configuration.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4ag
mkdir -p $O
j() { grep -E '^\{' $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "pairs/s", d["ms_per_step"], "ms")'; }
X='blas@\(768, 81, 256, 3, 5, .*\);'
for r in a b c; do
  IIT_GEMM_EXCLUDE="$X" IIT_GEMM_REPORT=$O/decisions_x_$r.txt timeout -k 10 300 python3 -u bench.py > $O/bench_x_$r.log 2>&1 || { tail -30 $O/bench_x_$r.log; exit 1; }
  echo "no-blas tail $r: $(j bench_x_$r)"
  timeout -k 10 300 python3 -u bench.py > $O/bench_s_$r.log 2>&1 || { tail -30 $O/bench_s_$r.log; exit 1; }
  echo "shipped $r: $(j bench_s_$r)"
done
grep -E "768, 81, 256" $O/decisions_x_a.txt | head -5
IIT_GEMM_EXCLUDE="$X" timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o b -- python3 bench.py --steps 20 --warmup 3 > $O/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/prof.log; exit $rc; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -n 1)
python3 scripts/step_breakdown.py "$f" --steps 15 --top 120 --gaps 5 --dump-step $O/step_seq.txt > $O/step_breakdown.txt && head -3 $O/step_breakdown.txt
echo "Cijk rows: $(grep -c Cijk $O/step_breakdown.txt || true)"
rm -rf $O/prof
