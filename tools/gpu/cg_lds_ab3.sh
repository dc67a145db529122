# LDS CG three-way A/B on one box: Poisson tests on the new build, then the n=20/40/80 lines per library
#   gpurun -- bash tools/gpu/cg_lds_ab3.sh TAG LIB_A LIB_B   (the default build is "new")
set -o pipefail
T=${1:-cgl}
A=${2:-superresolution_for_pdes_amd/lib/dbg/libsrpde_cgold.so}
B=${3:-superresolution_for_pdes_amd/lib/dbg/libsrpde_cgdiv1.so}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_poisson.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/poisson_$T.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/poisson_$T.log; exit 1; }
tail -1 gpurun_out/poisson_$T.log
for L in a b new a b new; do
  case $L in a) export SRPDE_LIB=$A;; b) export SRPDE_LIB=$B;; new) unset SRPDE_LIB;; esac
  timeout -k 10 300 python bench.py --workload poisson --no-cpu-baseline --no-live-traffic --poisson-sizes 20:4096,40:1024,80:1024 > gpurun_out/bench_cgl_${T}_$L.json 2> gpurun_out/bench_cgl_$T.err || { echo "bench failed"; tail gpurun_out/bench_cgl_$T.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/bench_cgl_${T}_$L.json'))
print('$L', {k: (v['ms_per_batch'], v['mean_iters'], v['fp64_frac']) for k, v in d['config']['levels'].items()})"
done
