# Whole GPU suite + smoke + default bench line on one MI355X box.
#   gpurun -- bash tools/gpu/full.sh TAG     (logs under gpurun_out/)
set -o pipefail
T=${1:-full}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 180 --timeout-method thread -m gpu > gpurun_out/pytest_$T.log 2>&1 || { echo "pytest failed"; grep -v amdgpu gpurun_out/pytest_$T.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_$T.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_$T.log; exit 1; }
tail -1 gpurun_out/smoke_$T.log
timeout -k 10 400 python bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || { echo "bench failed"; tail -20 gpurun_out/bench_$T.err; exit 1; }
cat gpurun_out/bench_$T.json
