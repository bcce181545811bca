# Round 4: after removing the split-store GEMM candidate and the adjacency-based QKV bias packing: bounds-checked poison
# runs (incl. the LN-xhat16 backward), staged-backward test with xhat16, primed-training test detail, DP ZeRO-1
# breakdown, eval kernel stats.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4k
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then tail -20 $O/$name.log; exit $rc; fi
  return 0
}
IIT_CHECK_BOUNDS=1 step poison_bounds 300 python3 -u scripts/diag_uninit_poison.py --focused; grep -E "^\[bisect\]|Error" $O/poison_bounds.log | cut -c1-300
step poison_sweep 600 python3 -u scripts/diag_uninit_poison.py; grep -E "MISMATCH|differ" $O/poison_sweep.log | cut -c1-300 | head -40
IIT_LN_XHAT16=1 step staged_xhat16 300 python3 -u -m pytest tests/test_paired.py tests/test_hip_kernels.py -q -m gpu -k "staged or layernorm" --timeout 120 --timeout-method thread; tail -3 $O/staged_xhat16.log
step primed 400 python3 -u -m pytest tests/test_eval_graphs_gpu.py -x -q -m gpu --tb=long --timeout 300 --timeout-method thread; grep -E "Error|assert|^E " $O/primed.log | head -30; tail -3 $O/primed.log
IIT_ZERO=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29571 IIT_DP_FORCE_REDUCER=1 \
  step dp_prof_z1 400 rocprofv3 --kernel-trace --output-format csv -d $O/dpprof1 -o dp -- python3 bench.py --steps 20 --warmup 3
f=$(find $O/dpprof1 -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 15 --top 30 --gaps 6 > $O/dp_breakdown_z1.txt && head -34 $O/dp_breakdown_z1.txt
rm -rf $O/dpprof1
step ioi_ckpt 300 python3 -u train_ioi.py --model gpt2-small --dtype bf16 --epochs 2 --num-samples 4000 --save-root /tmp/r4models --no-early-stop
step eval_prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/evprof -o ev -- python3 eval_ioi.py --model gpt2-small -w 100_100_40 --root /tmp/r4models --backend hip --num-samples 4608 --timing-repeats 1
grep -E "eval_ioi_timing" $O/eval_prof.log | cut -c1-300
f=$(find $O/evprof -name "*kernel_stats.csv" | head -n 1)
[ -n "$f" ] && head -25 "$f" | cut -c1-200 > $O/eval_kernel_stats.txt && cat $O/eval_kernel_stats.txt
rm -rf $O/evprof
du -sh gpurun_out
