# Run GPU tests on one MI355X box:  gpurun -- bash tools/gpu/tests.sh TAG [pytest selectors...]
# (default selector: the whole -m gpu suite).  Log under gpurun_out/pytest_TAG.log.
set -o pipefail
T=${1:-t}
shift
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
SEL=${@:-tests}
timeout -k 10 900 python -u -m pytest $SEL -x -v --timeout 180 --timeout-method thread -m gpu > gpurun_out/pytest_$T.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_$T.log | grep -v amdgpu | tail -60
exit $rc
