# Round 4: in-context re-tune of the GEMM decision table after the transposed epilogue, bench A/B new vs shipped.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4m
mkdir -p $O
IIT_GEMM_TABLE=0 timeout -k 10 700 python3 -u scripts/tune_gemm_in_situ.py --out $O/table_insitu.json \
  --report $O/insitu_report.txt > $O/tune.log 2>&1 || { echo tune failed; tail -30 $O/tune.log; exit 1; }
tail -3 $O/tune.log
j() { grep -E '^\{' $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "pairs/s", d["ms_per_step"], "ms")'; }
for r in a b; do
  IIT_GEMM_TABLE=$O/table_insitu.json timeout -k 10 300 python3 -u bench.py > $O/bench_new_$r.log 2>&1 || { tail -30 $O/bench_new_$r.log; exit 1; }
  echo "new $r: $(j bench_new_$r)"
  timeout -k 10 300 python3 -u bench.py > $O/bench_shipped_$r.log 2>&1 || { tail -30 $O/bench_shipped_$r.log; exit 1; }
  echo "shipped $r: $(j bench_shipped_$r)"
done
