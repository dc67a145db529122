# Stream-priority A/B of the train step and the DataParallel (RCCL) path under torchrun.
set -o pipefail
T=${1:-s16}
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_${T}_a.json 2> gpurun_out/bench_${T}_a.err || { echo "bench a failed"; exit 1; }
SRPDE_BWD_PRIORITY=1 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_${T}_prio.json 2> gpurun_out/bench_${T}_prio.err || { echo "bench prio failed"; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_${T}_b.json 2> gpurun_out/bench_${T}_b.err || { echo "bench b failed"; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 1 --steps 10 --warmup 3 --ddp --no-cpu-baseline > gpurun_out/bench_${T}_ddp.json 2> gpurun_out/bench_${T}_ddp.err || { echo "ddp failed"; tail -20 gpurun_out/bench_${T}_ddp.err; exit 1; }
for f in a prio b ddp; do echo "$f: $(python -c "import json,sys; d=json.load(open('gpurun_out/bench_${T}_$f.json')); print(d['ms_per_step'], d['value'], d['config'].get('parallelism'))")"; done
