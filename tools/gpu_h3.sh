# h3 bring-up on one MI355X: kernel tests (incl. fp64 accuracy), per-layer conv bench h3 vs x6
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
T=${1:-h3}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -s --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_$T.log 2>&1 || { echo "pytest failed"; grep -v amdgpu gpurun_out/pytest_$T.log | tail -40; exit 1; }
grep "fp64 errors" gpurun_out/pytest_$T.log; tail -1 gpurun_out/pytest_$T.log
timeout -k 10 200 python tools/conv_bench.py --math h3 > gpurun_out/convbench_${T}.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/convbench_${T}.log; exit 1; }
grep -v amdgpu gpurun_out/convbench_${T}.log
echo done
