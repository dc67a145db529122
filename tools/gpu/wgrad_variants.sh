# Weight-gradient timing of diagnostic / candidate builds (lib/dbg/lib<NAME>.so; "intree" = the tree's build):
#   gpurun -- bash tools/gpu/wgrad_variants.sh TAG LAYERS TESTED_NAME NAME...
set -o pipefail
T=$1; L=$2; TN=$3; shift 3
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
if [ "$TN" != none ]; then
  SRPDE_LIB=$R/superresolution_for_pdes_amd/lib/dbg/lib$TN.so timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_b1024.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/wv_${T}.log 2>&1 || { echo "tests failed"; grep -v amdgpu gpurun_out/wv_${T}.log | tail -20; exit 1; }
  tail -1 gpurun_out/wv_${T}.log
fi
for rep in 1 2; do
for V in intree "$@"; do
  L2=$R/superresolution_for_pdes_amd/lib/dbg/lib$V.so
  [ "$V" = intree ] && L2=$R/superresolution_for_pdes_amd/lib/libsrpde_hip.so
  echo "== $V ($rep)"
  SRPDE_LIB=$L2 timeout -k 10 200 python tools/conv_bench.py --only wgrad --layers $L --iters 10 2>&1 | grep -v amdgpu | grep -v "^TOTAL\|^#" || exit 1
done
done
