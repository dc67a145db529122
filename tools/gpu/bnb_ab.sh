# Isolated BN-backward-apply A/B (tools/bnb_bench.py) of library variants, interleaved on one box,
# then the train step A/B of the baseline (lib/ab/libsrpde_hip_base.so) against the tree's build.
#   gpurun -- bash tools/gpu/bnb_ab.sh TAG "VARIANT.so ..." [STEP_REPS]
set -o pipefail
T=${1:-bnb}
V=${2:-}
N=${3:-0}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
for rep in 1 2; do
  for v in base new $V; do
    case $v in
      base) export SRPDE_LIB=$R/superresolution_for_pdes_amd/lib/ab/libsrpde_hip_base.so ;;
      new) unset SRPDE_LIB ;;
      *) export SRPDE_LIB=$R/superresolution_for_pdes_amd/lib/ab/$v ;;
    esac
    echo "== $v $rep"
    timeout -k 10 120 python tools/bnb_bench.py --iters 20 2>&1 | grep -v amdgpu || exit 1
  done
done
unset SRPDE_LIB
if [ "$N" -gt 0 ]; then bash tools/gpu/step_ab.sh $T $N; fi
