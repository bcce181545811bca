#!/bin/bash
# ZeRO-1 with graph-captured DP phases and deferred gathers, two gloo ranks sharing one GPU:
# checksum / loss agreement with the replicated run (bench.py self-launch, weak scaling)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6x
mkdir -p $O
for z in 0 1; do
  IIT_ZERO=$z IIT_REHEARSE_ONE_GPU=1 IIT_DIST_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --steps 5 --warmup 2 > $O/zero$z.log 2>&1 || { echo "zero=$z failed"; tail -30 $O/zero$z.log; exit 5; }
  echo "zero=$z: $(grep -E '^\{' $O/zero$z.log | grep -o '"ms_per_step": [0-9.]*\|"last_train_losses": {[^}]*}' | tr '\n' ' ')"
done
IIT_ZERO=1 IIT_ZERO_POISON=1 IIT_REHEARSE_ONE_GPU=1 IIT_DIST_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --steps 5 --warmup 2 > $O/zero1_poison.log 2>&1 || { echo "poison failed"; tail -30 $O/zero1_poison.log; exit 6; }
echo "zero=1 poisoned: $(grep -E '^\{' $O/zero1_poison.log | grep -o '"ms_per_step": [0-9.]*\|"last_train_losses": {[^}]*}' | tr '\n' ' ')"
