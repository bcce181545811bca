# Round 4 (session 2): fourth in-context re-tune at HEAD (ragged tails on the repo's kernels), A/B x3 vs the shipped table
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4ai
mkdir -p $O
j() { grep -E '^\{' $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "pairs/s", d["ms_per_step"], "ms")'; }
export IIT_GEMM_EXCLUDE='blas@\(\d+, 2304, 768, 2, 1, True, False, False\);'
IIT_GEMM_TABLE=0 timeout -k 10 800 python3 -u scripts/tune_gemm_in_situ.py --out $O/table_insitu.json \
  --report $O/insitu_report.txt --top 8 --rounds 24 > $O/tune.log 2>&1 || { echo tune failed; tail -30 $O/tune.log; exit 1; }
tail -3 $O/tune.log
unset IIT_GEMM_EXCLUDE
for r in a b c; do
  IIT_GEMM_TABLE=$O/table_insitu.json IIT_GEMM_REPORT=$O/decisions_new_$r.txt timeout -k 10 300 python3 -u bench.py > $O/bench_new_$r.log 2>&1 || { tail -30 $O/bench_new_$r.log; exit 1; }
  echo "new $r: $(j bench_new_$r)"
  timeout -k 10 300 python3 -u bench.py > $O/bench_shipped_$r.log 2>&1 || { tail -30 $O/bench_shipped_$r.log; exit 1; }
  echo "shipped $r: $(j bench_shipped_$r)"
done
grep -c "blas" $O/decisions_new_a.txt || true
