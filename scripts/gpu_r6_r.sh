#!/bin/bash
# in-step vs isolated time per GEMM problem (isolated autotune: IIT_GEMM_TABLE=0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6r
mkdir -p $O
timeout -k 10 600 env IIT_GEMM_TABLE=0 python3 -u scripts/gemm_context_penalty.py > $O/penalty.log 2>&1 || { echo failed; tail -30 $O/penalty.log; exit 1; }
grep -v "amdgpu.ids" $O/penalty.log | head -60
