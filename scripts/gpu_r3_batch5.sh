# Round 3 batch 5: duplicate-node learnability vs learning rate (per-node IIT loss tracked).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3e
run() {
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/r3e/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; grep -E '^\{' "gpurun_out/r3e/$name.log" | tail -1 | cut -c1-700
  if [ $rc -ge 124 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
  return 0
}
run dup_lr1e-4 300 python3 -u scripts/iia_ceiling.py --epochs 30 --every 5 --train-nodes hook_duplicate
run dup_lr1e-3 300 python3 -u scripts/iia_ceiling.py --epochs 30 --every 5 --train-nodes hook_duplicate --lr 1e-3
run all_lr1e-3 300 python3 -u scripts/iia_ceiling.py --epochs 30 --every 5 --lr 1e-3
echo "batch done"
