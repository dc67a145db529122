# Forward / dgrad timing of diagnostic h4 builds (lib/dbg/lib<NAME>.so; "intree" = the tree's build):
#   gpurun -- bash tools/gpu/h4_variants.sh TAG LAYERS PASSES NAME...
set -o pipefail
T=$1; L=$2; K=$3; shift 3
R=$GRAFT_REPO_ROOT
cd $R
for V in intree "$@"; do
  L2=$R/superresolution_for_pdes_amd/lib/dbg/lib$V.so
  [ "$V" = intree ] && L2=$R/superresolution_for_pdes_amd/lib/libsrpde_hip.so
  echo "== $V"
  SRPDE_LIB=$L2 timeout -k 10 200 python tools/conv_bench.py --only $K --layers $L --iters 10 2>&1 | grep -v amdgpu | grep -v "^TOTAL\|^#" || exit 1
done
