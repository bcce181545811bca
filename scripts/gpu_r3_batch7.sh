# Round 3 batch 7: paired/splice GPU tests; train.py's full MNIST-PVR configuration (60k/10k, 10 epochs) wall clock;
# eval_ioi sweep timing on the HIP engine (cold + warm) and the fp32 torch-op backend; one-step kernel sequence.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3h
run() {
  local name=$1 secs=$2; shift 2
  echo "== $name"
  local t0=$(date +%s.%N)
  timeout -k 10 "$secs" "$@" > "gpurun_out/r3h/$name.log" 2>&1
  local rc=$?
  local t1=$(date +%s.%N)
  echo "   rc=$rc wall_s=$(python3 -c "print(round($t1-$t0,1))")"; grep -v amdgpu.ids "gpurun_out/r3h/$name.log" | tail -3 | cut -c1-500
  if [ $rc -ge 124 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
  return 0
}
run tests_paired 400 python3 -u -m pytest tests/test_paired.py tests/test_splice.py -x -q --timeout 120 --timeout-method thread
run train_py_full 900 python3 -u train.py
run ioi_ckpt 300 python3 -u train_ioi.py --model gpt2-small --dtype bf16 --epochs 2 --num-samples 4000 --save-root /tmp/r3models --no-early-stop
run eval_ioi_hip 600 python3 -u eval_ioi.py --model gpt2-small -w 100_100_40 --root /tmp/r3models --backend hip --num-samples 4608 --timing-repeats 2
run eval_ioi_torch 900 python3 -u eval_ioi.py --model gpt2-small -w 100_100_40 --root /tmp/r3models --backend torch --num-samples 4608
run step_trace 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3h/st -o st -- python3 -u bench.py --steps 20 --warmup 5
f=$(find gpurun_out/r3h/st -name "*kernel_trace.csv" | head -n 1)
python3 scripts/step_breakdown.py "$f" --steps 15 --top 60 --dump-step gpurun_out/r3h/one_step.txt > gpurun_out/r3h/step_breakdown.txt; rm -f "$f"
echo "batch done"
