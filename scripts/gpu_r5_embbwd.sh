set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5eb; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py -k "embed" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/b$i.log 2>&1 || exit 1; grep -o '"ms_per_step": [0-9.]*' $O/b$i.log; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o b -- python3 bench.py --steps 10 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -n 1)
[ -n "$f" ] && grep -i "embed_bwd\|pos_bwd" "$f" | cut -c1-200
rm -rf $O/prof
