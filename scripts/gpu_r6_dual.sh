#!/bin/bash
# Dual dX + dW pairs: in-step vs isolated vs prefix cache states (timing), then two counter passes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6dual
mkdir -p $O
timeout -k 10 300 python3 -u scripts/dual_l2_probe.py > $O/time.log 2>&1 || { echo time failed; tail -20 $O/time.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/p1 -o p -- python3 -u scripts/dual_l2_probe.py --pmc --seq $O/seq1.json > $O/p1.log 2>&1 || { echo pass1 failed; tail -20 $O/p1.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT TCC_MISS TCC_EA0_RDREQ TCC_EA0_WRREQ GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/p2 -o p -- python3 -u scripts/dual_l2_probe.py --pmc --seq $O/seq2.json > $O/p2.log 2>&1 || { echo pass2 failed; tail -20 $O/p2.log; exit 1; }
for p in 1 2; do
  f=$(ls $O/p$p/*counter_collection.csv 2>/dev/null | head -1)
  [ -n "$f" ] || f=$(find $O/p$p -name '*counter_collection.csv' | head -1)
  python3 scripts/dual_l2_probe.py --summarize "$f" --seq $O/seq$p.json > $O/sum$p.txt 2>&1 || echo "summary $p failed"
  find $O/p$p -name '*.csv' -size +20M -delete
done
cat $O/time.log | tail -12
cat $O/sum1.txt $O/sum2.txt
# MQNLI: op sites, then the traced breakdown and the untraced step with the library-free shipped table
timeout -k 10 300 python3 -u scripts/op_sites.py --family mqnli-bert-base > $O/mq_sites.txt 2>&1 || { echo sites failed; tail -20 $O/mq_sites.txt; exit 1; }
head -45 $O/mq_sites.txt
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/mqprof -o mq -- python3 scripts/bench_families.py --family mqnli-bert-base --steps 12 --warmup 3 > $O/mq_prof.log 2>&1 || { tail -20 $O/mq_prof.log; exit 1; }
f=$(find $O/mqprof -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 8 --top 40 --gaps 5 > $O/mqnli_breakdown.txt && head -50 $O/mqnli_breakdown.txt; rm -f "$f"
for r in 1 2; do
  timeout -k 10 300 python3 -u scripts/bench_families.py --family mqnli-bert-base --steps 30 --warmup 5 > $O/mq$r.log 2>&1 || { echo mq failed; tail -20 $O/mq$r.log; exit 1; }
  echo "mqnli: $(grep -E '^\{' $O/mq$r.log | cut -c1-200)"
done
