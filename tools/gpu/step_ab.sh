# Train-step A/B on ONE box: the baseline library (tools/build_base.sh -> lib/ab/libsrpde_hip_base.so,
# selected with SRPDE_LIB) against the tree's build, interleaved; optional test selector first.
#   gpurun -- bash tools/gpu/step_ab.sh TAG [REPS] [PYTEST_K]
set -o pipefail
T=${1:-ab}
N=${2:-3}
K=${3:-}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 500 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "$K" > gpurun_out/stepab_pytest_$T.log 2>&1 || { echo "tests failed"; grep -v amdgpu gpurun_out/stepab_pytest_$T.log | tail -30; exit 1; }
  tail -1 gpurun_out/stepab_pytest_$T.log
fi
for rep in $(seq 1 $N); do
  for v in base new; do
    if [ $v = base ]; then export SRPDE_LIB=$R/superresolution_for_pdes_amd/lib/ab/libsrpde_hip_base.so; else unset SRPDE_LIB; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-live-traffic --steps 20 > gpurun_out/stepab_${T}_${v}_$rep.json 2> gpurun_out/stepab_${T}_${v}_$rep.err || { echo "bench $v failed"; tail gpurun_out/stepab_${T}_${v}_$rep.err; exit 1; }
    echo "$v $rep $(python -c "import json; d=json.load(open('gpurun_out/stepab_${T}_${v}_$rep.json')); print(d['ms_per_step'], d['value'])")"
  done
done
