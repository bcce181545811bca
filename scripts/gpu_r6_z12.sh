#!/bin/bash
# precision study, second seed: 6L/64d seed 1, 300 epochs, whole-split IIA every 50 -- fp32 torch-op oracle vs HIP bf16
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6z12
mkdir -p $O
for be in torch hip; do
  timeout -k 10 560 python3 -u scripts/iia_ceiling.py --model ioi-6l --epochs 300 --every 50 --seed 1 --backend $be > $O/6l_s1_${be}_300.log 2>&1 || { tail -20 $O/6l_s1_${be}_300.log; exit 1; }
  echo "== $be"; grep -E '^Epoch (50|100|150|200|250|299):' $O/6l_s1_${be}_300.log | cut -c1-150
  grep -E '"metric"' $O/6l_s1_${be}_300.log | cut -c300-700
done
