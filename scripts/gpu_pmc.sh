# Hardware-counter passes over the step's main GEMM kernels (scripts/pmc_gemm.py): MFMA busy cycles, LDS bank
# conflicts, L2 hit / miss.  Counters only with --kernel-trace (no trace domains), one pass per counter group.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc1 gpurun_out/pmc2
timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc1 -o p -- python3 scripts/pmc_gemm.py > gpurun_out/pmc1/run.log 2>&1 || { echo pass1 failed; tail -5 gpurun_out/pmc1/run.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT TCC_MISS TCC_EA0_RDREQ TCC_EA0_WRREQ GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc2 -o p -- python3 scripts/pmc_gemm.py > gpurun_out/pmc2/run.log 2>&1 || { echo pass2 failed; tail -5 gpurun_out/pmc2/run.log; exit 1; }
find gpurun_out/pmc1 gpurun_out/pmc2 -name "*counter_collection.csv" | head
