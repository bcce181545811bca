#!/bin/bash
# Llama-3-8B S=512 step at HEAD: paired (torch backend) vs two forwards
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6w
mkdir -p $O
for p in 1 0; do
  timeout -k 10 500 env IIT_PAIRED_TORCH=$p python3 -u scripts/bench_families.py --family llama3-8b-causal --seq 512 --steps 5 --warmup 2 > $O/llama_p$p.log 2>&1 || { echo llama failed; tail -30 $O/llama_p$p.log; exit 1; }
  echo "llama paired=$p: $(grep -E '^\{' $O/llama_p$p.log | grep -o '"ms_per_step": [0-9.]*\|"peak_mem_gb": [0-9.]*' | tr '\n' ' ')"
done
