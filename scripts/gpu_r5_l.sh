#!/bin/bash
# Round 5: Llama-3-8B S=512 step at HEAD (flash-store hook_z splice, tiles 40/41 among the dW candidates) + kernel breakdown;
# MQNLI post-fix kernel breakdown
set -o pipefail
O=gpurun_out/r5l; mkdir -p $O
timeout -k 10 500 python3 -u scripts/bench_families.py --family llama3-8b-causal --seq 512 --steps 5 --warmup 2 > $O/llama.log 2>&1 || { tail -30 $O/llama.log; exit 1; }
grep -E '^\{' $O/llama.log | cut -c1-300
grep -E "^\[gemm\]" $O/llama.log | sort | uniq -c | sort -rn | head -20
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/mqprof -o mq -- python3 scripts/bench_families.py --family mqnli-bert-base --steps 12 --warmup 3 > $O/mq_prof.log 2>&1 || { tail -20 $O/mq_prof.log; exit 1; }
grep -E '^\{' $O/mq_prof.log | cut -c1-200
f=$(find $O/mqprof -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 8 --top 40 --gaps 5 > $O/mqnli_breakdown.txt && head -30 $O/mqnli_breakdown.txt; rm -f "$f"
timeout -k 10 400 python3 -u scripts/bench_families.py --family mqnli-bert-base --steps 30 --warmup 5 > $O/mq.log 2>&1 || { tail -20 $O/mq.log; exit 1; }
grep -E '^\{' $O/mq.log | cut -c1-250
