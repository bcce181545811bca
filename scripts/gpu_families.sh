# the other BASELINE model families at HEAD (1 GPU): MQNLI <-> BERT-base and the causal graph <-> Llama-3-8B
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fam
timeout -k 10 400 python scripts/bench_families.py --family mqnli-bert-base --steps 10 --warmup 3 > gpurun_out/fam/bert.log 2>&1 || { echo bert failed $?; tail -20 gpurun_out/fam/bert.log; exit 3; }
tail -1 gpurun_out/fam/bert.log
timeout -k 10 600 python scripts/bench_families.py --family llama3-8b-causal --steps 5 --warmup 2 > gpurun_out/fam/llama.log 2>&1 || { echo llama failed $?; tail -20 gpurun_out/fam/llama.log; exit 4; }
tail -1 gpurun_out/fam/llama.log
