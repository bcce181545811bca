# Round 3 batch 8: does the bf16 gradient wire change the IIA trajectory?  The 1-rank forced-reducer DP path
# (RCCL, IIT_DP_FORCE_REDUCER=1) on GPT-2-small for 62 epochs with the fp32 and the bf16 wire, and with ZeRO-1.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3i
run() {
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/r3i/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; grep -E '^\{' "gpurun_out/r3i/$name.log" | tail -1 | cut -c1-700
  if [ $rc -ge 124 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
  return 0
}
IIT_GEMM_TABLE=0 run llama_gemm_study 600 python3 -u scripts/llama_gemm_study.py
TR="python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1"
IIT_DP_FORCE_REDUCER=1 IIT_DP_GRAD_DTYPE=fp32 run wire_fp32 400 $TR --master-port 29521 scripts/time_to_iia.py --model gpt2-small --dtype bf16 --epochs 62
IIT_DP_FORCE_REDUCER=1 IIT_DP_GRAD_DTYPE=bf16 run wire_bf16 400 $TR --master-port 29522 scripts/time_to_iia.py --model gpt2-small --dtype bf16 --epochs 62
IIT_DP_FORCE_REDUCER=1 IIT_ZERO=1 run zero1_fp32 400 $TR --master-port 29523 scripts/time_to_iia.py --model gpt2-small --dtype bf16 --epochs 62
# train-loop vs bench gap: roctx phase ranges of 6 training epochs (epoch 0 = autotune + captures)
IIT_PROFILE=1 run loop_markers 400 rocprofv3 --marker-trace --output-format csv -d gpurun_out/r3i/mk -o mk -- python3 -u scripts/time_to_iia.py --model gpt2-small --dtype bf16 --epochs 6
f=$(find gpurun_out/r3i/mk -name "*marker_api_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/marker_summary.py "$f" > gpurun_out/r3i/loop_markers.txt; rm -f gpurun_out/r3i/mk/*trace.csv
echo "batch done"
