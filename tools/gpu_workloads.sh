# config #3 (Poisson CG) and config #5 (cascade) bench lines + kernel-trace stats of each
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
T=${1:-wl}
timeout -k 10 300 python -m pytest tests/test_gpu_cascade.py tests/test_gpu_poisson.py -x -q -m gpu > gpurun_out/pytest_$T.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_$T.log; exit 1; }
tail -1 gpurun_out/pytest_$T.log
timeout -k 10 300 python bench.py --workload poisson --steps 10 > gpurun_out/bench_poisson_$T.json 2> gpurun_out/bench_poisson_$T.err || { echo "poisson bench failed"; tail -20 gpurun_out/bench_poisson_$T.err; exit 1; }
cat gpurun_out/bench_poisson_$T.json
timeout -k 10 300 python bench.py --workload cascade --steps 10 --warmup 2 > gpurun_out/bench_cascade_$T.json 2> gpurun_out/bench_cascade_$T.err || { echo "cascade bench failed"; tail -20 gpurun_out/bench_cascade_$T.err; exit 1; }
cat gpurun_out/bench_cascade_$T.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_poisson_$T -o poisson -- python $R/bench.py --workload poisson --steps 3 --no-cpu-baseline > /dev/null 2>&1 || { echo "prof poisson failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_cascade_$T -o cascade -- python $R/bench.py --workload cascade --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>&1 || { echo "prof cascade failed"; exit 1; }
echo done
