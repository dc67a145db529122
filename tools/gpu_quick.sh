set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_unet.py -x -q -m gpu > gpurun_out/pytest_quick.log 2>&1; echo "pytest rc=$?"
timeout -k 10 200 python tools/conv_bench.py --only ${1:-fwd} > gpurun_out/convbench_quick.log 2>&1; echo "bench rc=$?"
