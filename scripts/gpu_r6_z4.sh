#!/bin/bash
# GPT-2-small on the fp32 torch-op oracle (graph-captured), 150 epochs, whole-split per-node IIA every 25: does fp32
# learn hook_duplicate where the HIP bf16 engine stays at ~1 % (profiles/iia_gpt2_1000_r6.txt)?
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6z
mkdir -p $O
timeout -k 10 1150 python3 -u scripts/iia_ceiling.py --model gpt2-small --epochs 150 --every 25 --seed 0 --backend torch > $O/gpt2_s0_torch_150.log 2>&1 || { tail -20 $O/gpt2_s0_torch_150.log; exit 1; }
grep -E '"metric"' $O/gpt2_s0_torch_150.log | cut -c1-420
