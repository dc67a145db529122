# backward stream-priority A/B (interleaved) + schedule tests
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
T=${1:-s10}
timeout -k 10 300 python -u -m pytest tests/test_gpu_schedule.py tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_$T.log 2>&1 || { echo "pytest failed"; grep -v amdgpu gpurun_out/pytest_$T.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_$T.log
for pr in 0 1 0 1; do
  SRPDE_BWD_PRIORITY=$pr timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_${T}_p$pr.json 2> gpurun_out/bench_${T}_p$pr.err || { echo "bench failed"; tail -20 gpurun_out/bench_${T}_p$pr.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_${T}_p$pr.json'));print('prio=$pr',d['ms_per_step'],d['value'],d['roofline']['launch_ms'])"
done
echo done
