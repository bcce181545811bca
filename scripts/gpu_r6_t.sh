#!/bin/bash
# re-tune the headline decision table in context with the dual-pair prefetch on, merge into the shipped table, A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6t
mkdir -p $O
timeout -k 10 600 env IIT_GEMM_TABLE=0 python3 -u scripts/tune_gemm_in_situ.py --out $O/table_new.json --report $O/report.txt --rounds 16 > $O/tune.log 2>&1 || { echo tune failed; tail -30 $O/tune.log; exit 1; }
tail -3 $O/tune.log
python3 - <<'PY'
import json
old = json.load(open("iit_amd/ops/tuned/gemm_decisions_gfx950.json"))
new = json.load(open("gpurun_out/r6t/table_new.json"))
changed = {k: (old["decisions"].get(k), v) for k, v in new["decisions"].items() if old["decisions"].get(k) != v}
old["decisions"].update(new["decisions"])
json.dump(old, open("gpurun_out/r6t/table_merged.json", "w"), indent=0, sort_keys=True)
print(len(changed), "decisions changed:")
for k, (a, b) in sorted(changed.items()):
    print(" ", k, a, "->", b)
PY
for k in 1 2; do
  for t in default merged; do
    if [ $t = merged ]; then tab=$O/table_merged.json; else tab=iit_amd/ops/tuned/gemm_decisions_gfx950.json; fi
    timeout -k 10 200 env IIT_GEMM_TABLE=$tab python3 -u bench.py --gpus 1 --steps 40 --warmup 5 > $O/b_$t.$k.log 2>&1 || { echo bench failed; tail -20 $O/b_$t.$k.log; exit 1; }
    echo "table $t: $(grep -E '^\{' $O/b_$t.$k.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
