#!/bin/bash
# Round 5: headline gradient precision split test, IIA-ceiling control (zero-W_O) on both engines
set -o pipefail
mkdir -p gpurun_out/r5c
timeout -k 10 300 python -u -m pytest tests/test_headline_parity.py -q -s --timeout 280 --timeout-method thread > gpurun_out/r5c/parity.log 2>&1; echo "parity rc=$?"
timeout -k 10 300 python -u scripts/iia_ceiling.py --model gpt2-small --epochs 30 --every 5 --control zero-wo > gpurun_out/r5c/ctl_gpt2_hip.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/iia_ceiling.py --model ioi-6l --epochs 100 --every 20 --control zero-wo > gpurun_out/r5c/ctl_6l_hip.log 2>&1 || exit 1
timeout -k 10 400 python -u scripts/iia_ceiling.py --model ioi-6l --epochs 100 --every 20 --control zero-wo --backend torch --graphs 0 > gpurun_out/r5c/ctl_6l_torch.log 2>&1 || exit 1
