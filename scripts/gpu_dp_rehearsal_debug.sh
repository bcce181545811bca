# Debug variant of gpu_dp_rehearsal.sh: two gloo ranks on cuda:0 started directly (no torchrun), each dumping every
# thread's Python stack after 100 s (faulthandler) if it has not finished -- to locate a hang.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export IIT_REHEARSE_ONE_GPU=1 IIT_DIST_BACKEND=gloo MASTER_ADDR=127.0.0.1 MASTER_PORT=29544 WORLD_SIZE=2
export IIT_BENCH_STREAM_CTX=${IIT_BENCH_STREAM_CTX:-1}
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r timeout -k 10 160 python -X faulthandler -c "
import faulthandler, sys, runpy
faulthandler.dump_traceback_later(100, exit=True)
sys.argv = ['bench.py', '--gpus', '2', '--steps', '4', '--warmup', '3']
runpy.run_path('bench.py', run_name='__main__')
" > gpurun_out/dbg_rank$r.log 2>&1 &
done
wait
echo done
