# Round-end confirmation: whole GPU suite + smoke (tools/gpu_round.sh without the PMC passes),
# the end-to-end data-gen + training + cascade accuracy run.
set -o pipefail
T=${1:-final}
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_$T.log 2>&1 || { echo "pytest failed"; grep -v amdgpu gpurun_out/pytest_$T.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_$T.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_$T.log; exit 1; }
tail -1 gpurun_out/smoke_$T.log
timeout -k 10 400 python -u tools/e2e_accuracy.py > gpurun_out/e2e_$T.log 2>&1 || { echo "e2e failed"; tail -20 gpurun_out/e2e_$T.log; exit 1; }
tail -3 gpurun_out/e2e_$T.log
echo done
