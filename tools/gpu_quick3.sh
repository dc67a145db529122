# kernel/unet GPU tests, conv micro-bench, HBM traffic PMC for a few layers (fwd)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
T=${1:-q3}
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_unet.py -x -q -m gpu > gpurun_out/pytest_$T.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_$T.log; exit 1; }
timeout -k 10 200 python tools/conv_bench.py --only ${2:-fwd,dgrad} > gpurun_out/convbench_$T.log 2>&1 || { echo "bench failed"; exit 1; }
cd /tmp
for L in bridge.3 enc2.conv2 dec1.conv1; do
  i=0
  for C in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/gpurun_out/pmc_${T}_$L -o p$i -- python $R/tools/conv_bench.py --layers $L --only fwd --iters 3 > /dev/null 2>&1 || { echo "pmc $L $C failed"; exit 1; }
  done
done
echo done
