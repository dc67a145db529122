# h3h weight-gradient timing: the shipped library against a diagnostic build (SRPDE_LIB), interleaved
#   gpurun -- bash tools/gpu/h3h_dbg.sh LIB [LAYERS]
set -o pipefail
L=$1; LAY=${2:-enc1.conv2,dec1.conv1,dec1.conv2,out_conv1}
R=$GRAFT_REPO_ROOT
cd $R
for rep in 1 2; do
  echo "== shipped $rep"; timeout -k 10 120 python tools/conv_bench.py --only wgrad --layers $LAY --iters 10 2>&1 | grep -v amdgpu || exit 1
  echo "== $L $rep"; SRPDE_LIB=$R/$L timeout -k 10 120 python tools/conv_bench.py --only wgrad --layers $LAY --iters 10 2>&1 | grep -v amdgpu || exit 1
done
