# A/B on one box: XCD tile-order group height 8 (round-2/3 order) vs the row-major default, interleaved.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3v
git_table=iit_amd/ops/tuned/gemm_decisions_gfx950.json
for rep in 1 2; do
  for gm in 8 0; do
    IIT_GEMM_GROUP_M=$gm timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > gpurun_out/r3v/b_gm${gm}_$rep.log 2>&1 || exit 1
    echo "gm=$gm rep=$rep $(grep -h '^{' gpurun_out/r3v/b_gm${gm}_$rep.log | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
