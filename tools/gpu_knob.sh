# kernel tests, then the fwd/dgrad conv bench for each value of an env knob
# usage: bash tools/gpu_knob.sh TAG KNOB "v1 v2 ..." [conv_bench args]
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
T=$1; KNOB=$2; VALS=$3; shift 3
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_$T.log 2>&1 || { echo "pytest failed"; grep -v amdgpu gpurun_out/pytest_$T.log | tail -40; exit 1; }
tail -1 gpurun_out/pytest_$T.log
for V in $VALS; do
  echo "== $KNOB=$V"
  env $KNOB=$V timeout -k 10 200 python tools/conv_bench.py "$@" > gpurun_out/convbench_${T}_$V.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/convbench_${T}_$V.log; exit 1; }
  grep -v amdgpu gpurun_out/convbench_${T}_$V.log
done
echo done
