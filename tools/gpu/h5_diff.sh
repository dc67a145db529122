# h5 vs h4 mismatch map for candidate builds:  gpurun -- bash tools/gpu/h5_diff.sh "N H C0 C1 COUT" NAME...
set -o pipefail
A=$1; shift
R=$GRAFT_REPO_ROOT
cd $R
for V in "$@"; do
  echo "== $V"
  L=$R/superresolution_for_pdes_amd/lib/dbg/lib$V.so
  [ "$V" = intree ] && L=$R/superresolution_for_pdes_amd/lib/libsrpde_hip.so
  SRPDE_LIB=$L timeout -k 10 120 python -u tools/h5_diff.py $A 2>&1 | grep -v amdgpu || exit 1
done
