# Row-blocked upsample backward: GPU tests, isolated A/B against the pixel-blocked gather, bench.
set -o pipefail
T=${1:-s14}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_unet.py tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_$T.log 2>&1 || { echo "pytest failed"; grep -v amdgpu gpurun_out/pytest_$T.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_$T.log
timeout -k 10 200 python tools/pw_bench.py > gpurun_out/pw_rows_$T.log 2>&1 || { echo "pw failed"; tail gpurun_out/pw_rows_$T.log; exit 1; }
SRPDE_UPSAMPLE_BWD=px timeout -k 10 200 python tools/pw_bench.py > gpurun_out/pw_px_$T.log 2>&1 || { echo "pw px failed"; exit 1; }
grep upsample gpurun_out/pw_rows_$T.log gpurun_out/pw_px_$T.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || { echo "bench failed"; tail -20 gpurun_out/bench_$T.err; exit 1; }
cat gpurun_out/bench_$T.json
SRPDE_UPSAMPLE_BWD=px timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_${T}_px.json 2> gpurun_out/bench_${T}_px.err || { echo "bench px failed"; exit 1; }
cat gpurun_out/bench_${T}_px.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$T -o bench -- python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_$T.log 2>&1 || { echo "prof failed"; exit 1; }
echo done
