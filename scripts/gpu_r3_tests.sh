# Round 3: the full GPU test tier (as the driver runs it), then the bench.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_gpu_r3.log 2>&1
rc=$?
tail -25 gpurun_out/pytest_gpu_r3.log
exit $rc
