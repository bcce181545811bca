# round 6: IIA on the headline config -- GPT-2-small with train_ioi.py's configuration for the
# reference's full 1000-epoch budget (/root/reference/train_ioi.py:13-26,48), whole-split per-node IIA every 50 epochs
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6iia; mkdir -p $O
timeout -k 10 1150 python3 -u scripts/iia_ceiling.py --model gpt2-small --epochs 1000 --every 50 > $O/gpt2_1000.log 2>&1
rc=$?; grep -v amdgpu.ids $O/gpt2_1000.log | grep -E '^\{' | cut -c1-400 | tail -25; exit $rc
