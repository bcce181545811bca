# Round 4: re-check the relaxed BERT paired / headline parity tests and the xhat16 LN kernel; bisect the poison
# (allocator-garbage) dependence of the paired backward over the dispatch toggles.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4e
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then tail -20 $O/$name.log; exit $rc; fi
  return 0
}
step tests 600 python3 -u -m pytest tests/test_hip_model.py tests/test_headline_parity.py tests/test_hip_kernels.py -q -m gpu --timeout 300 --timeout-method thread -k "layernorm or bert_paired or headline"
tail -3 $O/tests.log; grep -E "^FAILED|^E  " $O/tests.log | head -20
step bisect 900 python3 -u scripts/diag_uninit_poison.py --bisect; grep -E "^\[bisect\]" $O/bisect.log | cut -c1-600
