# Round 4 (session 2): Llama-3-8B family on the native op kernels -- vectorised rotary / SwiGLU / RMSNorm-dw
# (IIT_LLAMA_VEC=0: the previous kernels), the residual-add GEMM epilogue and the RMSNorm fork (IIT_TORCH_RESID_EPI /
# IIT_RMS_FORK), S = 512; then a kernel breakdown of the default configuration.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4o
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -30 $O/$name.log; exit $rc; fi
  return 0
}
jf() { grep -E '^\{' $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], d["ms_per_step"], "ms", "peak", d.get("peak_mem_gb"))'; }
step llama_tests 300 python3 -u -m pytest tests/test_llama_ops.py -q -m gpu --timeout 120 --timeout-method thread
tail -1 $O/llama_tests.log
F="scripts/bench_families.py --family llama3-8b-causal --seq 512 --steps 4 --warmup 2"
IIT_LLAMA_VEC=0 IIT_TORCH_RESID_EPI=0 IIT_RMS_FORK=0 step ll_old 600 python3 -u $F; jf ll_old
IIT_TORCH_RESID_EPI=0 IIT_RMS_FORK=0 step ll_vec 600 python3 -u $F; jf ll_vec
IIT_TORCH_RESID_EPI=1 IIT_RMS_FORK=1 step ll_fused 600 python3 -u $F; jf ll_fused
IIT_TORCH_RESID_EPI=1 IIT_RMS_FORK=1 step ll_prof 900 rocprofv3 --kernel-trace --output-format csv -d $O/llprof -o ll -- python3 $F
f=$(find $O/llprof -name "*kernel_trace.csv" | head -n 1)
[ -n "$f" ] && python3 scripts/step_breakdown.py "$f" --steps 3 --top 40 --gaps 3 > $O/llama_breakdown.txt && head -50 $O/llama_breakdown.txt
rm -rf $O/llprof
IIT_EVAL_GRAPHS=0 step eval_profile 600 python3 -u scripts/profile_eval.py
grep -E "^\[eval\]" $O/eval_profile.log
