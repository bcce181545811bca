# round 6, call D: implicit-GEMM conv tests + microbench, BN reduction A/B (microbench, PVR step), the torch-backend
# paired forward (Llama tests), the Llama-3-8B S=512 step with the paired forward on / off
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6d; mkdir -p $O
for red in two atomic; do
  IIT_BN_REDUCE=$red timeout -k 10 200 python3 scripts/bench_bn.py > $O/bn_$red.log 2>&1 || { tail -20 $O/bn_$red.log; exit 3; }
  echo "== bn $red"; grep -E '^\{' $O/bn_$red.log
done
for cfg in "two 1" "two 0" "atomic 0"; do
  set -- $cfg
  IIT_BN_REDUCE=$1 IIT_CONV_HIP=$([ $2 = 1 ] && echo auto || echo 0) timeout -k 10 300 python3 scripts/bench_families.py --family pvr-resnet18 --dtype bf16 --steps 20 --warmup 3 > $O/pvr_$1_$2.log 2>&1 || { tail -20 $O/pvr_$1_$2.log; exit 4; }
  echo "pvr bn=$1 conv=$2: $(grep -E '^\{' $O/pvr_$1_$2.log | cut -c1-160)"
done
for pt in 1 0; do
  IIT_PAIRED_TORCH=$pt timeout -k 10 500 python3 scripts/bench_families.py --family llama3-8b-causal --seq 512 --steps 4 --warmup 2 > $O/llama_paired$pt.log 2>&1 || { tail -20 $O/llama_paired$pt.log; exit 5; }
  echo "llama paired=$pt: $(grep -E '^\{' $O/llama_paired$pt.log | cut -c1-260)"
done
