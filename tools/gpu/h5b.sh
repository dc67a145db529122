# h5 tests + A/B (layers, forward) + diagnostic variant libraries (lib/dbg/libh5dbg*.so):
#   gpurun -- bash tools/gpu/h5b.sh TAG
set -o pipefail
T=${1:-h5}
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu/h5.sh $T || exit $?
for LIB in superresolution_for_pdes_amd/lib/dbg/libh5*.so; do
  echo "== $LIB"
  SRPDE_LIB=$R/$LIB timeout -k 10 200 python -u tools/h5_ab.py --layers --reps 1 2>&1 | grep -v amdgpu | grep "h5=1" || exit 1
done
