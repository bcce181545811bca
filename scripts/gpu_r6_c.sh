# round 6, call C: BatchNorm statistics (pivot-shifted sums; two-level partials + finalize vs round 5's atomics +
# ticket: tests, per-layer microbench A/B, PVR bf16 step A/B), the torch-backend paired forward (Llama tests), then
# the Llama-3-8B S=512 step with the paired forward on / off
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_bn_fused.py tests/test_llama_ops.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert|FAILED" $O/pytest.log | head -30; tail -30 $O/pytest.log; exit $rc; }
for red in two atomic; do
  IIT_BN_REDUCE=$red timeout -k 10 200 python3 scripts/bench_bn.py > $O/bn_$red.log 2>&1 || { tail -20 $O/bn_$red.log; exit 2; }
  echo "== bn $red"; grep -E '^\{' $O/bn_$red.log
  IIT_BN_REDUCE=$red timeout -k 10 300 python3 scripts/bench_families.py --family pvr-resnet18 --dtype bf16 --steps 20 --warmup 3 > $O/pvr_$red.log 2>&1 || { tail -20 $O/pvr_$red.log; exit 2; }
  grep -E '^\{' $O/pvr_$red.log | cut -c1-200
done
for pt in 1 0; do
  IIT_PAIRED_TORCH=$pt timeout -k 10 500 python3 scripts/bench_families.py --family llama3-8b-causal --seq 512 --steps 4 --warmup 2 > $O/llama_paired$pt.log 2>&1 || { tail -20 $O/llama_paired$pt.log; exit 3; }
  echo "paired=$pt: $(grep -E '^\{' $O/llama_paired$pt.log | cut -c1-260)"
done
