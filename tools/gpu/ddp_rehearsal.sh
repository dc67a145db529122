# Rehearse bench.py's N > 1 path on ONE GPU: 2 ranks over gloo (RCCL refuses two ranks on one
# device), DataParallel gradient buckets, barriers, max-over-ranks timing.
#   gpurun -- bash tools/gpu/ddp_rehearsal.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export SRPDE_BENCH_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 3 --warmup 2 --batch 256 --no-cpu-baseline > gpurun_out/ddp_rehearsal.json 2> gpurun_out/ddp_rehearsal.err || { echo "rehearsal failed"; tail -30 gpurun_out/ddp_rehearsal.err; exit 1; }
cat gpurun_out/ddp_rehearsal.json
