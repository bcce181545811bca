# Flash-attention check on the GPU box: parity tests, then the microbenchmark with the automatic and the forced
# query-block policies (IIT_FLASH_QB).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for qb in 1 2; do  # both block-per-wave variants of every kernel (the automatic policy picks by grid size)
  IIT_FLASH_QB=$qb timeout -k 10 300 python -u -m pytest tests/test_flash_attn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_flash$qb.log 2>&1 || { tail -30 gpurun_out/pt_flash$qb.log; exit 1; }
  echo "IIT_FLASH_QB=$qb: $(tail -1 gpurun_out/pt_flash$qb.log)"
done
for qb in 0 1 2; do
  IIT_FLASH_QB=$qb timeout -k 10 200 python scripts/bench_flash.py > gpurun_out/flash_qb$qb.txt 2>&1 || exit 3
  echo "IIT_FLASH_QB=$qb"; cat gpurun_out/flash_qb$qb.txt
done
