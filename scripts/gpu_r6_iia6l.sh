# round 6: the 6L/64d reference model's plateau exit, 2 seeds x {HIP bf16, fp32 torch-op oracle}, 150 epochs each
# (quantify the engine divergence seen in profiles/iia_ceiling_r5.txt:19-37)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6iia6; mkdir -p $O
for seed in 0 1; do
  for be in hip torch; do
    timeout -k 10 420 python3 -u scripts/iia_ceiling.py --model ioi-6l --epochs 150 --every 10 --seed $seed --backend $be \
      > $O/6l_s${seed}_$be.log 2>&1 || { tail -20 $O/6l_s${seed}_$be.log; exit 1; }
    echo "seed $seed $be: $(grep -E '"metric"' $O/6l_s${seed}_$be.log | cut -c1-300)"
  done
done
# the vs_baseline denominator at HEAD (it was a 5-step round-1 run): the reference-semantics eager
# engine (hook closures, full-vocab fp32 logits, torch Adam), 20 timed steps
timeout -k 10 300 python3 bench.py --engine reference --dtype fp32 --graphs 0 --steps 20 --warmup 3 > $O/ref_eager.log 2>&1 \
  || { tail -20 $O/ref_eager.log; exit 2; }
grep -E '^\{' $O/ref_eager.log | cut -c1-300
