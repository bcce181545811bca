# Where do the LDS-DMA GEMM tiles wait?  Four counter passes (one per run, --kernel-trace only) over scripts/pmc_gemm.py.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3r
pass() {
  local n=$1; shift
  mkdir -p gpurun_out/r3r/p$n
  timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/r3r/p$n -o p -- python3 scripts/pmc_gemm.py > gpurun_out/r3r/p$n.log 2>&1
  local rc=$?
  echo "pass $n rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/r3r/p$n.log; return $rc; }
}
pass 1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE || exit 1
pass 2 SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE || exit 1
pass 3 TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_UTCL1_TRANSLATION_MISS TCP_PENDING_STALL_CYCLES GRBM_GUI_ACTIVE || exit 1
pass 4 TCC_HIT TCC_MISS TCC_EA0_RDREQ GRBM_GUI_ACTIVE || exit 1
python3 scripts/pmc_deep_summary.py $(find gpurun_out/r3r -name "*counter_collection.csv") > gpurun_out/r3r/summary.txt
find gpurun_out/r3r -name "*.csv" -delete
head -80 gpurun_out/r3r/summary.txt
