# cooperative CG A/B (round 4): tests, then bench per block size through SRPDE_GCG_NPT_TMP -- a temporary
# override in srpde_poisson_cg_batched, removed after the A/B (profiles/r04q_poisson_npt.txt)
#   gpurun -- bash tools/gpu/cg2.sh TAG
set -o pipefail
T=${1:-cg2}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_poisson.py tests/test_gpu_cascade.py tests/test_gpu_poisson_rows.py tests/test_gpu_report.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/poisson_$T.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/poisson_$T.log; exit 1; }
tail -1 gpurun_out/poisson_$T.log
run() {  # V sizes tag
  SRPDE_GCG_NPT_TMP=$1 timeout -k 10 300 python bench.py --workload poisson --no-cpu-baseline --poisson-sizes $2 > gpurun_out/bench_poisson_${T}_$3.json 2> gpurun_out/bench_poisson_$T.err || { echo "bench failed"; tail gpurun_out/bench_poisson_$T.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/bench_poisson_${T}_$3.json'))
print('$3', {k: (v['B'], v['ms_per_batch'], v['mean_iters']) for k, v in d['config']['levels'].items()})"
}
for V in 2 4 8; do
  env -u SRPDE_GCG_NPT_TMP true
  run $V 160:1,320:1,640:1 b1_$V || exit 1
done
unset SRPDE_GCG_NPT_TMP
timeout -k 10 300 python bench.py --workload poisson --no-cpu-baseline > gpurun_out/bench_poisson_${T}_def.json 2>> gpurun_out/bench_poisson_$T.err || exit 1
cut -c1-1500 gpurun_out/bench_poisson_${T}_def.json
