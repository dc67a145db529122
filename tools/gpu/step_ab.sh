# Same-box step A/B of the in-tree library against lib/ab/libsrpde_hip_base.so (tools/build_base.sh, tools/build_variant_git.sh), after the
# GPU tests named by PYTEST_K.   gpurun -- bash tools/gpu/step_ab.sh TAG [REPS] [PYTEST_K]
set -o pipefail
T=${1:-lab}
N=${2:-3}
K=${3:-}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu -k "$K" > gpurun_out/lab_pytest_$T.log 2>&1 || { echo "tests failed"; grep -v amdgpu gpurun_out/lab_pytest_$T.log | tail -30; exit 1; }
  tail -1 gpurun_out/lab_pytest_$T.log
fi
for rep in $(seq 1 $N); do
  for v in base new; do
    if [ $v = base ]; then export SRPDE_LIB=$R/superresolution_for_pdes_amd/lib/ab/libsrpde_hip_base.so; else unset SRPDE_LIB; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-live-traffic --steps 20 --warmup 3 > gpurun_out/lab_${T}_${v}_$rep.json 2> gpurun_out/lab_${T}_${v}_$rep.err || { echo "bench $v failed"; tail gpurun_out/lab_${T}_${v}_$rep.err; exit 1; }
    echo "$v $rep $(python -c "import json; d=json.load(open('gpurun_out/lab_${T}_${v}_$rep.json')); print(d['ms_per_step'], d['value'])")"
  done
done
