# Round 4 (session 2): training wall-clock at HEAD (scripts/time_to_iia.py, every phase graph primed before epoch 0)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4ae
mkdir -p $O
timeout -k 10 400 python3 -u scripts/time_to_iia.py --model gpt2-small --dtype bf16 --epochs 80 > $O/tti_gpt2.log 2>&1
rc=$?; echo "gpt2 rc=$rc"; grep -E "primed|^\{" $O/tti_gpt2.log | cut -c1-700; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u scripts/time_to_iia.py --model ioi-6l --dtype bf16 --epochs 150 > $O/tti_6l.log 2>&1
rc=$?; echo "6l rc=$rc"; grep -E "primed|^\{" $O/tti_6l.log | cut -c1-700
