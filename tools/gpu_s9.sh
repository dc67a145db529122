# cascade graphs: GPU tests, cascade bench, train bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
T=${1:-s9}
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_$T.log 2>&1 || { echo "pytest failed"; grep -v amdgpu gpurun_out/pytest_$T.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_$T.log
timeout -k 10 300 python bench.py --workload cascade > gpurun_out/bench_${T}_cascade.json 2> gpurun_out/bench_${T}_cascade.err || { echo "cascade bench failed"; tail -20 gpurun_out/bench_${T}_cascade.err; exit 1; }
cut -c1-900 gpurun_out/bench_${T}_cascade.json
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_${T}.json 2> gpurun_out/bench_${T}.err || { echo "bench failed"; tail -20 gpurun_out/bench_${T}.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_${T}.json'));print(d['ms_per_step'],d['value'],d['roofline']['launch_ms'])"
echo done
