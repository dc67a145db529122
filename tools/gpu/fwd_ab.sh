# Eval / train forward A/B of a candidate build (lib/dbg/lib<NAME>.so) against the tree's, interleaved, with an
# optional pytest -k run on the candidate first:  gpurun -- bash tools/gpu/fwd_ab.sh TAG NAME [PYTEST_K]
set -o pipefail
T=$1; V=$2; K=${3:-}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
L2=$R/superresolution_for_pdes_amd/lib/dbg/lib$V.so
if [ -n "$K" ]; then
  SRPDE_LIB=$L2 timeout -k 10 400 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "$K" > gpurun_out/fwdab_$T.log 2>&1 || { echo "tests failed"; grep -v amdgpu gpurun_out/fwdab_$T.log | tail -20; exit 1; }
  tail -1 gpurun_out/fwdab_$T.log
fi
for rep in 1 2 3; do
  for v in base new; do
    if [ $v = new ]; then export SRPDE_LIB=$L2; else unset SRPDE_LIB; fi
    for m in eval train; do
      echo "$v $rep $m $(timeout -k 10 200 python tools/fwd_bench.py --mode $m 2>/dev/null | tail -1)"
    done
  done
done
