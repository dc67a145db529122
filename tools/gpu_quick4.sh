# conv GPU tests + conv micro-bench of all three passes (A/B of wgrad kernels)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
T=${1:-q4}
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_unet.py -x -q -m gpu > gpurun_out/pytest_$T.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_$T.log; exit 1; }
tail -1 gpurun_out/pytest_$T.log
timeout -k 10 200 python tools/conv_bench.py --only wgrad > gpurun_out/convbench_${T}_v2.log 2>&1 || { echo "bench failed"; exit 1; }
SRPDE_WGRAD64=1 timeout -k 10 200 python tools/conv_bench.py --only wgrad > gpurun_out/convbench_${T}_v2w.log 2>&1 || { echo "bench failed"; exit 1; }
SRPDE_WGRAD_V2=0 timeout -k 10 200 python tools/conv_bench.py --only wgrad > gpurun_out/convbench_${T}_v1.log 2>&1 || { echo "bench failed"; exit 1; }
echo done
