# Poisson: tests, block-size A/B at B=1 (override through the test hook), the config #3 line with live PMC
#   gpurun -- bash tools/gpu/r04q.sh TAG
set -o pipefail
T=${1:-r04q}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_poisson.py tests/test_gpu_cascade.py tests/test_gpu_poisson_rows.py tests/test_gpu_report.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/poisson_$T.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/poisson_$T.log; exit 1; }
tail -1 gpurun_out/poisson_$T.log
timeout -k 10 400 python bench.py --workload poisson > gpurun_out/bench_poisson_$T.json 2> gpurun_out/bench_poisson_$T.err || { echo "bench failed"; tail gpurun_out/bench_poisson_$T.err; exit 1; }
cat gpurun_out/bench_poisson_$T.json
timeout -k 10 300 python bench.py --workload poisson --no-cpu-baseline --no-live-traffic --poisson-sizes 160:1,320:1,640:1 > gpurun_out/bench_poisson_b1_$T.json 2>> gpurun_out/bench_poisson_$T.err || exit 1
python -c "
import json; d=json.load(open('gpurun_out/bench_poisson_b1_$T.json'))
print({k: (v['B'], v['ms_per_batch'], v['us_per_iter']) for k, v in d['config']['levels'].items()})"
