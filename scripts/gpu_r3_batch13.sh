# Round 3 batch 13: row-major XCD tile order -> GEMM tests, bench with the shipped table, in-context re-tune, bench.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3u
timeout -k 10 300 python3 -u -m pytest tests/test_gemm_glds.py tests/test_gemm_dispatch.py tests/test_hip_model.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3u/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r3u/tests.log; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > gpurun_out/r3u/bench_oldtable.log 2>&1 || exit 1
grep -E '^\{' gpurun_out/r3u/bench_oldtable.log | cut -c1-200
IIT_GEMM_TABLE=0 timeout -k 10 900 python3 -u scripts/tune_gemm_in_situ.py --out gpurun_out/r3u/gemm_decisions_in_situ.json \
  --report gpurun_out/r3u/gemm_in_situ_report.txt > gpurun_out/r3u/tune.log 2>&1 || { echo tune failed; tail -20 gpurun_out/r3u/tune.log; exit 1; }
cp gpurun_out/r3u/gemm_decisions_in_situ.json iit_amd/ops/tuned/gemm_decisions_gfx950.json
timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > gpurun_out/r3u/bench_newtable.log 2>&1 || exit 1
grep -E '^\{' gpurun_out/r3u/bench_newtable.log | cut -c1-200
timeout -k 10 300 python3 -u bench.py > gpurun_out/r3u/bench_default.log 2>&1 || exit 1
grep -E '^\{' gpurun_out/r3u/bench_default.log | cut -c1-200
