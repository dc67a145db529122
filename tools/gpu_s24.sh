# XCD-aware row order of the row-blocked upsample backward: kernel tests, isolated timing, one FETCH pass, bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_unet.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_s24.log 2>&1 || { echo "pytest failed"; grep -v amdgpu gpurun_out/pytest_s24.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_s24.log
timeout -k 10 200 python tools/pw_bench.py > gpurun_out/pw_s24.log 2>&1 || { echo "pw failed"; exit 1; }
grep upsample gpurun_out/pw_s24.log
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_s24 -o p1 -- python $R/tools/pw_bench.py --iters 2 > $R/gpurun_out/pmc_s24.log 2>&1 || { echo "pmc failed"; exit 1; }
cd $R
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_s24.json 2> gpurun_out/bench_s24.err || { echo "bench failed"; exit 1; }
SRPDE_UPSAMPLE_BWD=px timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_s24_px.json 2> gpurun_out/bench_s24_px.err || { echo "bench px failed"; exit 1; }
for f in s24 s24_px; do echo "$f: $(python -c "import json; d=json.load(open('gpurun_out/bench_$f.json')); print(d['ms_per_step'], d['value'])")"; done
