# grid CG three-way A/B on one box: the grid levels (and B=1) per library (default build = "new")
#   gpurun -- bash tools/gpu/grid_ab3.sh TAG LIB_A LIB_B
set -o pipefail
T=${1:-grid3}
A=$2
B=$3
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for L in new a b new a b; do
  case $L in a) export SRPDE_LIB=$A;; b) export SRPDE_LIB=$B;; new) unset SRPDE_LIB;; esac
  for S in 160:64,320:16,640:4 160:1,640:1; do
    timeout -k 10 300 python bench.py --workload poisson --no-cpu-baseline --no-live-traffic --poisson-sizes $S > gpurun_out/grid3_${T}_$L.json 2> gpurun_out/grid3_$T.err || { echo "bench failed"; tail gpurun_out/grid3_$T.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/grid3_${T}_$L.json'))
print('$L', {k: (v['B'], v['ms_per_batch'], v['us_per_iter']) for k, v in d['config']['levels'].items()})"
  done
done
