# round 5: 8-phase GEMM tests (both schedules), isolated bench, counter pass
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_8ph.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5b_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5b_tests.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/r5b_tests.log; exit $rc; }
timeout -k 10 600 python -u scripts/bench_gemm_8ph.py > gpurun_out/r5b_bench.log 2>&1
rc=$?; tail -15 gpurun_out/r5b_bench.log; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/pmc8
timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc8 -o p -- python3 scripts/pmc_8ph.py > gpurun_out/pmc8_run.log 2>&1 || { echo pmc failed; tail -5 gpurun_out/pmc8_run.log; exit 1; }
python3 scripts/pmc_8ph.py --summary $(find gpurun_out/pmc8 -name "*counter_collection.csv") > gpurun_out/pmc8_summary.txt; cat gpurun_out/pmc8_summary.txt
find gpurun_out/pmc8 -name "*counter_collection.csv" -delete
