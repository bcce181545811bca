#!/bin/bash
# precision study, seed 1 long runs: does either precision leave the plateau within the reference's budget?
#   $1 = torch (fp32 oracle, 800 epochs) | hip (bf16 engine, 1000 epochs); whole-split IIA every 100
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6z13
mkdir -p $O
be=$1; ep=$([ "$be" = torch ] && echo 800 || echo 1000)
timeout -k 10 1140 python3 -u scripts/iia_ceiling.py --model ioi-6l --epochs $ep --every 100 --seed 1 --backend $be > $O/6l_s1_${be}_$ep.log 2>&1 || { tail -20 $O/6l_s1_${be}_$ep.log; exit 1; }
grep -E '^Epoch (100|200|300|400|500|600|700|799|800|900|999):' $O/6l_s1_${be}_$ep.log | cut -c1-150
grep -E '"metric"' $O/6l_s1_${be}_$ep.log | cut -c300-800
