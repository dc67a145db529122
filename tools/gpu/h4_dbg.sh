# Phase ablation of the h4 kernel (timing-only builds: SRPDE_CONV_DBG bits make results wrong), each a
# separate library under lib/dbg/ (SRPDE_EXTRA_FLAGS=-DSRPDE_CONV_DBG=N SRPDE_BUILD_OUT=...):
#   1 no DMA in the taps, 2 no tap barrier, 4 no per-chunk convert, 16 no epilogue, 128 no MFMAs
#   gpurun -- bash tools/gpu/h4_dbg.sh [LAYERS]
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
L=${1:-bridge.3,dec3.conv1,dec2.conv1,enc2.conv2}
for D in ${H4_DBG:-0 1 2 4 16 128}; do
  echo "== dbg $D"
  if [ $D = 0 ]; then unset SRPDE_LIB; else export SRPDE_LIB=$R/superresolution_for_pdes_amd/lib/dbg/libsrpde_dbg$D.so; fi
  timeout -k 10 120 python tools/conv_bench.py --layers $L --only fwd,dgrad --iters 10 2>&1 | grep -v amdgpu || exit 1
done
unset SRPDE_LIB
