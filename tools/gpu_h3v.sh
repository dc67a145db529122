# h3 variants A/B on one MI355X: kernel tests, then fwd/dgrad conv bench with an env knob on/off
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
T=${1:-h3v}
KNOB=${2:-SRPDE_H3_RELAX}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -s --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_$T.log 2>&1 || { echo "pytest failed"; grep -v amdgpu gpurun_out/pytest_$T.log | tail -40; exit 1; }
grep "fp64 errors" gpurun_out/pytest_$T.log | cut -c1-220; tail -1 gpurun_out/pytest_$T.log
for V in 0 1; do
  echo "== $KNOB=$V"
  env $KNOB=$V timeout -k 10 200 python tools/conv_bench.py --only fwd,dgrad > gpurun_out/convbench_${T}_$V.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/convbench_${T}_$V.log; exit 1; }
  grep -v amdgpu gpurun_out/convbench_${T}_$V.log
done
echo done
