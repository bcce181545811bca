# Round 3 session 2 final validation at HEAD: full GPU suite, smoke, the driver's default bench, the 2-rank DP
# rehearsal (gloo, one GPU: dual launches / fused bias sums under the DP reducer), kernel trace of the headline step.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3s2z
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|FAIL|assert" $O/tests.log | head -30; exit $rc; }
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log | cut -c1-200
timeout -k 10 300 python3 -u bench.py > $O/bench_default.log 2>&1 || { tail -30 $O/bench_default.log; exit 1; }
grep -E '^\{' $O/bench_default.log
timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > $O/bench_100.log 2>&1 || { tail -30 $O/bench_100.log; exit 1; }
grep -E '^\{' $O/bench_100.log | cut -c1-200
export IIT_REHEARSE_ONE_GPU=1 IIT_DIST_BACKEND=gloo
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 4 --warmup 3 > $O/dp_rehearsal.log 2>&1 || { tail -30 $O/dp_rehearsal.log; exit 1; }
grep -E '^\{' $O/dp_rehearsal.log | cut -c1-200
unset IIT_REHEARSE_ONE_GPU IIT_DIST_BACKEND
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o st -- \
  python3 bench.py --steps 20 --warmup 3 > $O/bench_traced.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_trace.csv" | head -n 1)
python scripts/step_breakdown.py "$f" --steps 15 --top 70 --gaps 6 --dump-step $O/one_step.txt > $O/breakdown.txt && head -40 $O/breakdown.txt
rm -f "$f"
