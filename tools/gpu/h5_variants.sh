# layer times of diagnostic h5 builds (lib/dbg/libh5v<bits>.so, H5_DBG bits in conv_h5.hip):
#   gpurun -- bash tools/gpu/h5_variants.sh TAG BITS...
set -o pipefail
T=$1; shift
R=$GRAFT_REPO_ROOT
cd $R
for V in "$@"; do
  echo "== H5_DBG=$V"
  SRPDE_LIB=$R/superresolution_for_pdes_amd/lib/dbg/libh5v$V.so timeout -k 10 200 python -u tools/h5_ab.py --layers --reps 1 2>&1 | grep -v amdgpu | grep "h5=1" || exit 1
done
