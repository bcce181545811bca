# Round 3 batch 4: is the IOI duplicate node unlearnable, or does one engine path mis-train it?  Duplicate-only
# training on GPT-2-small: HIP engine with graphs, HIP engine eager, fp32 torch-op oracle backend.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3d
run() {
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/r3d/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; grep -E '^\{' "gpurun_out/r3d/$name.log" | tail -2 | cut -c1-500
  if [ $rc -ge 124 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
  return 0
}
run dup_graphs 300 python3 -u scripts/iia_ceiling.py --epochs 12 --every 3 --train-nodes hook_duplicate
run dup_eager 300 python3 -u scripts/iia_ceiling.py --epochs 12 --every 3 --train-nodes hook_duplicate --graphs 0
run dup_torch32 500 python3 -u scripts/iia_ceiling.py --epochs 12 --every 3 --train-nodes hook_duplicate --graphs 0 --backend torch
echo "batch done"
