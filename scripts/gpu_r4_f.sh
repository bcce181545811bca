set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4f
timeout -k 10 300 python3 -u scripts/diag_split_store.py > gpurun_out/r4f/split.log 2>&1; rc=$?
echo "== split rc=$rc"; grep -E "^\[split\]|Error|error" gpurun_out/r4f/split.log | head -40
if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then exit $rc; fi
bash scripts/gpu_r4_d.sh
