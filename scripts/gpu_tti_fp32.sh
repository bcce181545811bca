# Same-trajectory wall-clock comparison in fp32 (the engines agree to the printed digits in fp32): this engine
# (torch-op backend + graphs) vs the reference-semantics eager engine, GPT-2-small, train_ioi.py config
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tti
timeout -k 10 300 python -u scripts/time_to_iia.py --model gpt2-small --dtype fp32 --epochs 70 > gpurun_out/tti/gpt2_fp32_native.log 2>&1
rc=$?; tail -1 gpurun_out/tti/gpt2_fp32_native.log | cut -c1-700; [ $rc -eq 0 ] || exit $rc
timeout -k 10 800 python -u scripts/time_to_iia.py --model gpt2-small --dtype fp32 --engine reference --epochs 70 > gpurun_out/tti/gpt2_fp32_reference.log 2>&1
rc=$?; tail -1 gpurun_out/tti/gpt2_fp32_reference.log | cut -c1-700; exit $rc
