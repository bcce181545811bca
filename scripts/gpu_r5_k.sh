#!/bin/bash
# Round 5: PVR family step -- fp32 / bf16, fused BN on / off, MIOpen find mode on / off; kernel breakdown of the shipped bf16 step
set -o pipefail
O=gpurun_out/r5k; mkdir -p $O
run() { # name env...
  local n=$1; shift
  env "$@" timeout -k 10 400 python3 -u scripts/bench_families.py --family pvr-resnet18 --steps 20 --warmup 3 $EXTRA > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  echo "$n: $(grep -E '^\{' $O/$n.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"], "ms/step", r["value"], "pairs/s", "val_IIA", r["val_IIA"])')"
}
EXTRA=""; run fp32_find IIT_CONV_BENCHMARK=1
EXTRA=""; run fp32_nofind IIT_CONV_BENCHMARK=0
EXTRA="--dtype bf16"; run bf16_fused_find IIT_CONV_BENCHMARK=1 IIT_FUSED_BN=1
EXTRA="--dtype bf16"; run bf16_fused_nofind IIT_CONV_BENCHMARK=0 IIT_FUSED_BN=1
EXTRA="--dtype bf16"; run bf16_module_find IIT_CONV_BENCHMARK=1 IIT_FUSED_BN=0
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/pvrprof -o pvr -- python3 scripts/bench_families.py --family pvr-resnet18 --dtype bf16 --steps 10 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/pvrprof -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 6 --top 30 --gaps 3 > $O/pvr_bf16_breakdown.txt && head -12 $O/pvr_bf16_breakdown.txt; rm -f "$f"
