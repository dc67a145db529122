# h5 check on ONE box: the h5 tests, then the same-process A/B (per layer + whole forward).
#   gpurun -- bash tools/gpu/h5.sh TAG
set -o pipefail
T=${1:-h5}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_h5.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/h5_pytest_$T.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Error|assert" gpurun_out/h5_pytest_$T.log | grep -v amdgpu | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/h5_ab.py --layers --forward --reps 2 --json-out gpurun_out/h5_ab_$T.json 2>&1 | grep -v amdgpu | tee gpurun_out/h5_ab_$T.txt
