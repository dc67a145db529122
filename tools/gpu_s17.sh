# Kernel trace of the DataParallel train step at world 1 (single process, RCCL group of one).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_ddp -o bench -- python $R/bench.py --ddp --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_ddp.log 2>&1 || { echo "prof failed"; tail -20 $R/gpurun_out/prof_ddp.log; exit 1; }
echo done
