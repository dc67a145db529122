# One-GPU rehearsal of the RCCL path (verdict r4 #7): the plain step against DataParallel at world 1 under
# torch.distributed.run with the buckets' one-rank RCCL all-reduce kept (bench.py --ddp-rccl), interleaved
# on one box, then a kernel trace of each and its per-stream split.
#   gpurun -- bash tools/gpu/rccl_world1.sh TAG
set -o pipefail
T=${1:-rccl}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # $1 = plain|rccl, $2 = output stem, further args to bench.py
  local v=$1 o=$2; shift 2
  if [ $v = rccl ]; then
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port 29571 bench.py --gpus 1 --ddp-rccl --no-cpu-baseline --no-live-traffic "$@" > $o.json 2> $o.err
  else
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-live-traffic "$@" > $o.json 2> $o.err
  fi
}
for rep in 1 2 3; do
  for v in plain rccl; do
    run $v gpurun_out/w1_${T}_${v}_$rep --steps 20 --warmup 3 || { tail -5 gpurun_out/w1_${T}_${v}_$rep.err; exit 1; }
    echo "$v $rep $(python -c "import json; print(json.load(open('gpurun_out/w1_${T}_${v}_$rep.json'))['ms_per_step'])")"
  done
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/w1trace_${T}_plain -o bench -- python $R/bench.py --no-cpu-baseline --no-live-traffic --steps 8 --warmup 3 > $R/gpurun_out/w1trace_${T}_plain.log 2>&1 || { tail -5 $R/gpurun_out/w1trace_${T}_plain.log; exit 1; }
RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29572 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/w1trace_${T}_rccl -o bench -- python $R/bench.py --gpus 1 --ddp-rccl --no-cpu-baseline --no-live-traffic --steps 8 --warmup 3 > $R/gpurun_out/w1trace_${T}_rccl.log 2>&1 || { tail -5 $R/gpurun_out/w1trace_${T}_rccl.log; exit 1; }
cd $R
for v in plain rccl; do
  f=$(find gpurun_out/w1trace_${T}_$v -name "*kernel_trace.csv" | head -1)
  echo "== $v"; python tools/stream_split.py $f 6 | head -14
  echo "rccl kernels: $(grep -c -i "rccl\|nccl\|oneRank" $f)"
done
