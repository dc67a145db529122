# Poisson tests (spsolve fixtures, cooperative vs polled grid CG, cascade / report users) and the
# config #3 bench line:  gpurun -- bash tools/gpu/poisson_final.sh TAG
set -o pipefail
T=${1:-p}
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_poisson.py tests/test_gpu_cascade.py tests/test_gpu_poisson_rows.py tests/test_gpu_report.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/poisson_$T.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/poisson_$T.log; exit 1; }
tail -1 gpurun_out/poisson_$T.log
timeout -k 10 300 python bench.py --workload poisson > gpurun_out/bench_poisson_$T.json 2> gpurun_out/bench_poisson_$T.err || { echo "bench failed"; tail gpurun_out/bench_poisson_$T.err; exit 1; }
cat gpurun_out/bench_poisson_$T.json
timeout -k 10 300 python bench.py --workload poisson --no-cpu-baseline --poisson-sizes 640:1 > gpurun_out/bench_poisson640b1_$T.json 2>> gpurun_out/bench_poisson_$T.err || { echo "bench 640 failed"; exit 1; }
cat gpurun_out/bench_poisson640b1_$T.json
