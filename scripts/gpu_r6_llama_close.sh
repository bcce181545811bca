#!/bin/bash
# closing Llama-3-8B causal-graph step at HEAD (default: two forwards; S = 512, B = 16)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6fam
mkdir -p $O
timeout -k 10 600 python3 scripts/bench_families.py --family llama3-8b-causal --seq 512 --steps 4 --warmup 2 > $O/llama.log 2>&1 || { tail -20 $O/llama.log; exit 1; }
echo "llama: $(grep -E '^\{' $O/llama.log | grep -oE '"ms_per_step": [0-9.]+')"
