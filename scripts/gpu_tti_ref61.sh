# the reference-semantics eager engine (fp32) over the epochs this engine needs to reach val/IIA ~99.7 % (epoch 60)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tti
timeout -k 10 900 python -u scripts/time_to_iia.py --model gpt2-small --dtype fp32 --engine reference --epochs 61 > gpurun_out/tti/gpt2_fp32_reference.log 2>&1
rc=$?; grep -E "^Epoch (0|10|20|30|40|50|60):" gpurun_out/tti/gpt2_fp32_reference.log | cut -c1-170; tail -1 gpurun_out/tti/gpt2_fp32_reference.log | cut -c1-700; exit $rc
