# in-step GEMM hardware counters at round-6 closing HEAD (in-step MFMA busy; gemm_pmc_in_step_r6.txt)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6p; mkdir -p $O
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc -o p -- python3 -u bench.py --graphs 0 --steps 6 --warmup 3 > $O/pmc_run.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/pmc_run.log; exit 1; }
f=$(find $O/pmc -name "*counter_collection.csv" | head -n 1)
python3 scripts/pmc_step_summary.py "$f" 4 > $O/pmc_step_summary.txt; cat $O/pmc_step_summary.txt | tail -30
rm -rf $O/pmc
