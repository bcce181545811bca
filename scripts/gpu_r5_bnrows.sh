# fused BN kernels: row loops unrolled by 4; grid size A/B (IIT_BN_ROWS rows per thread group) on the PVR bf16 step
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5bn; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bn_fused.py > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for rows in 8 8; do
  IIT_BN_ROWS=$rows timeout -k 10 300 python3 -u scripts/bench_families.py --family pvr-resnet18 --dtype bf16 --steps 20 --warmup 3 > $O/pvr$rows.log 2>&1 || { tail -20 $O/pvr$rows.log; exit 1; }
  echo "rows=$rows $(grep -o '"ms_per_step": [0-9.]*' $O/pvr$rows.log)"
done
