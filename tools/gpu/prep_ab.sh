# weight-split preparation without per-element divisions: kernel tests, then the train step against the
# previous build (same box, alternating)
#   gpurun -- bash tools/gpu/prep_ab.sh TAG
set -o pipefail
T=${1:-prep}
OLD=superresolution_for_pdes_amd/lib/dbg/libsrpde_notailfuse.so
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/prep_tests_$T.log 2>&1 || { grep -v amdgpu gpurun_out/prep_tests_$T.log | tail -30; exit 1; }
tail -1 gpurun_out/prep_tests_$T.log
for L in old new old new; do
  if [ $L = old ]; then export SRPDE_LIB=$OLD; else unset SRPDE_LIB; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-live-traffic --steps 20 > gpurun_out/prep_bench_${T}_$L.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/prep_bench_${T}_$L.json')); print('$L', d['ms_per_step'])"
done
unset SRPDE_LIB
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prep_prof_$T -o b -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-live-traffic > /dev/null 2>&1 || exit 1
grep -i prepare_weights $GRAFT_REPO_ROOT/gpurun_out/prep_prof_$T/b_kernel_stats.csv | cut -c1-200
