#!/bin/bash
# round-6 late validation at HEAD (LN backward default R = 1, TorchOps bf16 emulation hooks): GPU tests, smoke, the
# driver's bench command; then the LN partial-reduce group A/B (scripts/gpu_r6_z9.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_final.sh || exit $?
bash scripts/gpu_r6_z9.sh
