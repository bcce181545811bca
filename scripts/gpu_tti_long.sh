# Long IOI training runs toward the reference's early-stop criterion (val/IIA = val/accuracy = 100):
# the reference's own IOI model (6L/64d, train_ioi.py config, up to its 1000-epoch budget) and GPT-2-small
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tti
timeout -k 10 540 python -u scripts/time_to_iia.py --model ioi-6l --dtype bf16 --epochs 1000 > gpurun_out/tti/ioi6l_bf16.log 2>&1
rc=$?; tail -1 gpurun_out/tti/ioi6l_bf16.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/time_to_iia.py --model gpt2-small --dtype bf16 --epochs 400 > gpurun_out/tti/gpt2_bf16.log 2>&1
rc=$?; tail -1 gpurun_out/tti/gpt2_bf16.log | cut -c1-600; exit $rc
