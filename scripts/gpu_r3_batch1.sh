# Round 3 batch: GPU tests, headline bench, IIA-ceiling analysis, PVR family bench, eval_ioi sweep timing,
# Llama-3-8B at S=512.  Each step has its own time limit; a test failure (rc 1) does not stop the batch, a fault /
# abort / time-out (rc >= 124) does.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/r3/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; grep -v amdgpu.ids "gpurun_out/r3/$name.log" | tail -3 | cut -c1-600
  if [ $rc -ge 124 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
  return 0
}
run pytest_gpu 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
run bench 300 python3 -u bench.py
run iia_ceiling 600 python3 -u scripts/iia_ceiling.py --epochs 70 --every 5
run pvr_fp32 400 python3 -u scripts/bench_families.py --family pvr-resnet18 --steps 10 --warmup 3
run ioi_ckpt 300 python3 -u train_ioi.py --model gpt2-small --dtype bf16 --epochs 2 --num-samples 4000 --save-root gpurun_out/r3/models --no-early-stop
run eval_ioi_hip 600 python3 -u eval_ioi.py --model gpt2-small -w 100_100_40 --root gpurun_out/r3/models --backend hip --num-samples 4608
run eval_ioi_torch 900 python3 -u eval_ioi.py --model gpt2-small -w 100_100_40 --root gpurun_out/r3/models --backend torch --num-samples 4608
run llama_s512 900 python3 -u scripts/bench_families.py --family llama3-8b-causal --seq 512 --steps 3 --warmup 1
echo "batch done"
