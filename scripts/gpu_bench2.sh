set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do
IIT_GEMM_REPORT=gpurun_out/gemm_decisions_$i.txt timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$i.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_$i.log; exit 5; }
tail -1 gpurun_out/bench_$i.log | cut -c1-220
done
