#!/bin/bash
# shipped ragged (unembed bulk + tail) decisions: GEMM tests, then the driver's bench twice with the decision report
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6z10
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gemm_glds.py tests/test_gemm_dispatch.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2; do
  IIT_GEMM_REPORT=$O/dec$i.txt timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/b$i.log 2>&1 || { tail -20 $O/b$i.log; exit 1; }
  echo "bench $i: $(tail -1 $O/b$i.log | grep -oE '"ms_per_step": [0-9.]+')  timed keys: $(grep '^M=' $O/dec$i.txt | grep -vc ' nan')"
done
