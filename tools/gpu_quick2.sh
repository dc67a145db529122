set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_unet.py -x -q -m gpu > gpurun_out/pytest_quick.log 2>&1; echo "pytest rc=$?"
SRPDE_CONV_TAIL=1 timeout -k 10 200 python tools/conv_bench.py --only fwd,dgrad > gpurun_out/convbench_tail1.log 2>&1; echo "bench rc=$?"
SRPDE_CONV_TAIL=0 timeout -k 10 200 python tools/conv_bench.py --only fwd,dgrad > gpurun_out/convbench_tail0.log 2>&1; echo "bench rc=$?"
