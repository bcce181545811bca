# round 5: root-cause experiment of the removed split-store GEMM candidate
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5ss
mkdir -p $O
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then tail -20 $O/$name.log; exit $rc; fi
  return 0
}
show() { grep -E "^\[bisect\]" $O/$1.log | sed 's/IIT_[A-Z_]*=[^ ]* //g' | awk -F'vs 0-last: ' '{n=split($2,a,", "); printf "%s | %d params differ | %s ... %s\n", $1, n, a[1], a[n]}'; }
export IIT_GEMM_SPLIT_STORE_KEY=32,128,512
for v in 1 atomic1 nosplit sync; do
  IIT_GEMM_SPLIT_STORE=$v step key_$v 300 python3 -u scripts/diag_uninit_poison.py --focused; show key_$v
done
