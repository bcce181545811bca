#!/bin/bash
# Round 5: flash-attention store splice tests, then the PVR leakiness sweep (fast vs per-node vs reference engine)
set -o pipefail
mkdir -p gpurun_out/r5f
timeout -k 10 300 python -u -m pytest tests/test_flash_attn.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r5f/flash.log 2>&1 || { tail -30 gpurun_out/r5f/flash.log; exit 1; }
tail -3 gpurun_out/r5f/flash.log
timeout -k 10 900 python -u scripts/eval_pvr_r4.py --engines native native_pernode reference --skip-info > gpurun_out/r5f/eval_pvr.log 2>&1
grep "\[pvr\]" gpurun_out/r5f/eval_pvr.log
