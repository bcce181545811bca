# counter passes incl. the reduction split-K GEMMs, then the tracing GPU test
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_pmc.sh || exit $?
p1=$(find gpurun_out/pmc1 -name "*counter_collection.csv" | head -n 1)
p2=$(find gpurun_out/pmc2 -name "*counter_collection.csv" | head -n 1)
python scripts/pmc_summary.py "$p1" "$p2" > gpurun_out/pmc_summary.txt && cat gpurun_out/pmc_summary.txt
rm -f "$p1" "$p2"
timeout -k 10 300 python -u -m pytest tests/test_tracing.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_tracing.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_tracing.log; exit $rc
