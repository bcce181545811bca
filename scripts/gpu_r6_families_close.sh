#!/bin/bash
# closing family numbers at HEAD: PVR ResNet-18 bf16 step and MQNLI BERT-base step (bench_families), 2 runs each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6fam
mkdir -p $O
for i in 1 2; do
  for fam in pvr-resnet18 mqnli-bert-base; do
    extra=""; [ "$fam" = pvr-resnet18 ] && extra="--dtype bf16"
    timeout -k 10 300 python3 -u scripts/bench_families.py --family $fam $extra --steps 20 --warmup 5 > $O/$fam.$i.log 2>&1 || { tail -20 $O/$fam.$i.log; exit 1; }
    echo "$fam $i: $(grep -E '^\{' $O/$fam.$i.log | grep -oE '"ms_per_step": [0-9.]+')"
  done
done
