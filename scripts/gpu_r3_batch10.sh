# Round 3 batch 10: fused IOI HL label kernel tests, IOI-path GPU tests, headline bench.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3l
timeout -k 10 600 python3 -u -m pytest tests/test_ioi_hl_kernel.py tests/test_paired.py tests/test_ioi_and_pairs.py tests/test_graphs.py tests/test_eval_ablations.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3l/tests.log 2>&1
rc=$?; tail -15 gpurun_out/r3l/tests.log; echo "rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > gpurun_out/r3l/bench.log 2>&1
rc=$?; grep -E '^\{' gpurun_out/r3l/bench.log | cut -c1-250; echo "rc=$rc"
