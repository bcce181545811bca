# fused LN affine-gradient backward (iit_ln_bwd_part): kernel tests, MQNLI / BERT tests, MQNLI step A/B
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5ln; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py tests/test_mqnli.py > $O/t.log 2>&1 \
  || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for f in 0 1; do
  IIT_LN_FUSED_DWDB=$f timeout -k 10 300 python3 -u scripts/bench_families.py --family mqnli-bert-base --steps 30 --warmup 5 > $O/mq$f.log 2>&1 || { tail -20 $O/mq$f.log; exit 1; }
  echo "fused=$f $(grep -o '"ms_per_step": [0-9.]*' $O/mq$f.log)"
done
IIT_LN_FUSED_DWDB=1 timeout -k 10 300 python3 -u scripts/bench_families.py --family mqnli-bert-base --steps 30 --warmup 5 > $O/mq1b.log 2>&1 || { tail -20 $O/mq1b.log; exit 1; }
echo "fused=1 (rep) $(grep -o '"ms_per_step": [0-9.]*' $O/mq1b.log)"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o mq -- python3 scripts/bench_families.py --family mqnli-bert-base --steps 12 --warmup 3 > $O/mq_prof.log 2>&1 || { tail -20 $O/mq_prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 8 --top 40 --gaps 5 > $O/mqnli_breakdown.txt && head -30 $O/mqnli_breakdown.txt | cut -c1-150; rm -rf $O/prof
