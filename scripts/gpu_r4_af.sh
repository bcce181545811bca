# Round 4 (session 2): full kernel list + one steady step's kernel sequence of the headline step at HEAD
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4af
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o b -- python3 bench.py --steps 20 --warmup 3 > $O/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/prof.log; exit $rc; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -n 1)
python3 scripts/step_breakdown.py "$f" --steps 15 --top 120 --gaps 12 --dump-step $O/step_seq.txt > $O/step_breakdown.txt && head -20 $O/step_breakdown.txt
rm -rf $O/prof
