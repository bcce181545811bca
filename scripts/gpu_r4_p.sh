# Round 4 (session 2): in-context re-tune of the GEMM decision table with hipBLASLt excluded from the packed-QKV
# forward (K03: the repo's LDS-DMA kernel on every QKV projection), then a same-box bench A/B against the shipped
# table (alternating, two rounds).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4p
mkdir -p $O
j() { grep -E '^\{' $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "pairs/s", d["ms_per_step"], "ms")'; }
export IIT_GEMM_EXCLUDE='blas@\(\d+, 2304, 768, 2, 1, True, False, False\);'
IIT_GEMM_TABLE=0 timeout -k 10 800 python3 -u scripts/tune_gemm_in_situ.py --out $O/table_insitu.json \
  --report $O/insitu_report.txt > $O/tune.log 2>&1 || { echo tune failed; tail -30 $O/tune.log; exit 1; }
tail -3 $O/tune.log
unset IIT_GEMM_EXCLUDE
for r in a b; do
  IIT_GEMM_TABLE=$O/table_insitu.json IIT_GEMM_REPORT=$O/decisions_new_$r.txt timeout -k 10 300 python3 -u bench.py > $O/bench_new_$r.log 2>&1 || { tail -30 $O/bench_new_$r.log; exit 1; }
  echo "new $r: $(j bench_new_$r)"
  timeout -k 10 300 python3 -u bench.py > $O/bench_shipped_$r.log 2>&1 || { tail -30 $O/bench_shipped_$r.log; exit 1; }
  echo "shipped $r: $(j bench_shipped_$r)"
done
grep -c "blas" $O/decisions_new_a.txt || true
# MQNLI <-> BERT-base step trace: the position splices run inside the LN kernel (no splice_kernel rows expected)
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mq -o mq -- python3 scripts/bench_families.py --family mqnli-bert-base --steps 12 --warmup 3 > $O/mq_run.log 2>&1
rc=$?; echo "mq prof rc=$rc"; grep -E '^\{' $O/mq_run.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
f=$(find $O/mq -name "*kernel_stats.csv" | head -n 1)
echo "splice rows in the MQNLI kernel stats: $(grep -ci splice "$f" || true)"
cp "$f" $O/mqnli_kernel_stats.csv
rm -rf $O/mq
