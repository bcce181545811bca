# Round 3 batch 11: executed FLOPs per headline step; in-step hardware counters of every GEMM dispatch.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3m/pmc
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/r3m/pmc -o p -- python3 -u bench.py --graphs 0 --steps 6 --warmup 3 > gpurun_out/r3m/pmc_run.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -2 gpurun_out/r3m/pmc_run.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/r3m/pmc -name "*counter_collection.csv" | head -n 1)
python3 scripts/pmc_step_summary.py "$f" 4 > gpurun_out/r3m/pmc_step_summary.txt; cat gpurun_out/r3m/pmc_step_summary.txt
rm -f gpurun_out/r3m/pmc/*.csv
