set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
T=${1:-x6p}
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q -m gpu > gpurun_out/pytest_$T.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_$T.log; exit 1; }
tail -1 gpurun_out/pytest_$T.log
timeout -k 10 200 python tools/conv_bench.py --only fwd,dgrad --math x6p > gpurun_out/convbench_${T}.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/convbench_${T}.log; exit 1; }
grep -v amdgpu gpurun_out/convbench_${T}.log
echo done
