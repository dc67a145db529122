# grid CG A/B on one box: Poisson tests on the new build, then the grid levels (and B=1) per library
#   gpurun -- bash tools/gpu/grid_ab.sh TAG OLD_LIB
set -o pipefail
T=${1:-grid}
OLD=${2:-superresolution_for_pdes_amd/lib/dbg/libsrpde_cgold.so}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_poisson.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/grid_$T.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/grid_$T.log; exit 1; }
tail -1 gpurun_out/grid_$T.log
for L in old new old new; do
  if [ $L = old ]; then export SRPDE_LIB=$OLD; else unset SRPDE_LIB; fi
  for S in 160:64,320:16,640:4 160:1,640:1; do
    timeout -k 10 300 python bench.py --workload poisson --no-cpu-baseline --no-live-traffic --poisson-sizes $S > gpurun_out/grid_${T}_$L.json 2> gpurun_out/grid_$T.err || { echo "bench failed"; tail gpurun_out/grid_$T.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/grid_${T}_$L.json'))
print('$L', {k: (v['B'], v['ms_per_batch'], v['us_per_iter']) for k, v in d['config']['levels'].items()})"
  done
done
