# Executor-choice A/B on ONE box (tools/bench_with.py: a module attribute set before bench.py runs), after the
# tests named by PYTEST_K.   gpurun -- bash tools/gpu/fuse_ab.sh TAG "ATTR=VALUE" [REPS] [PYTEST_K]
set -o pipefail
T=${1:-fab}
SETA=$2
N=${3:-2}
K=${4:-}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu -k "$K" > gpurun_out/fab_pytest_$T.log 2>&1 || { echo "tests failed"; grep -v amdgpu gpurun_out/fab_pytest_$T.log | tail -30; exit 1; }
  tail -1 gpurun_out/fab_pytest_$T.log
fi
for rep in $(seq 1 $N); do
  for v in base new; do
    if [ $v = base ]; then A="$SETA"; else A=""; fi
    timeout -k 10 200 python tools/bench_with.py $A -- --no-cpu-baseline --no-live-traffic --steps 20 > gpurun_out/fab_${T}_${v}_$rep.json 2> gpurun_out/fab_${T}_${v}_$rep.err || { echo "bench $v failed"; tail gpurun_out/fab_${T}_${v}_$rep.err; exit 1; }
    echo "$v $rep $(python -c "import json; d=json.load(open('gpurun_out/fab_${T}_${v}_$rep.json')); print(d['ms_per_step'], d['value'])")"
  done
done
