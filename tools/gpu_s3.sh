# Full GPU tests, the bench with the weight-gradient side stream on / off, and the phase split
# of the h3 forward / dgrad conv (SRPDE_CONV_DBG, timing only, results wrong: 16 = no epilogue,
# 1 = no DMA in the loop, 4 = no per-chunk split).
# usage: bash tools/gpu_s3.sh TAG     (outputs under gpurun_out/)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
T=${1:-s3}
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_$T.log 2>&1 || { echo "pytest failed"; grep -v amdgpu gpurun_out/pytest_$T.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_$T.log
for ws in 1 0; do
  SRPDE_WGRAD_STREAM=$ws timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_${T}_ws$ws.json 2> gpurun_out/bench_${T}_ws$ws.err || { echo "bench failed"; tail -20 gpurun_out/bench_${T}_ws$ws.err; exit 1; }
  echo "ws=$ws"; cat gpurun_out/bench_${T}_ws$ws.json
done
for d in 0 16 1 4; do
  SRPDE_CONV_DBG=$d timeout -k 10 200 python tools/conv_bench.py --only fwd,dgrad --iters 5 > gpurun_out/convbench_${T}_dbg$d.log 2>&1 || { echo "convbench failed"; tail gpurun_out/convbench_${T}_dbg$d.log; exit 1; }
  echo "dbg=$d"; cat gpurun_out/convbench_${T}_dbg$d.log
done
echo done
