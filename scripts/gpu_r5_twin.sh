# LN fp32 twin for post-norm residual operands (BERT): tests, MQNLI A/B
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5tw2; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py tests/test_mqnli.py tests/test_hip_model.py tests/test_paired.py > $O/t.log 2>&1 \
  || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for tw in 0 1 0 1; do
  IIT_LN_TWIN=$tw timeout -k 10 300 python3 -u scripts/bench_families.py --family mqnli-bert-base --steps 30 --warmup 5 > $O/mq$tw.log 2>&1 || { tail -20 $O/mq$tw.log; exit 1; }
  echo "twin=$tw $(grep -o '"ms_per_step": [0-9.]*\|"val_IIA": [0-9.]*' $O/mq$tw.log | tr '\n' ' ')"
done
