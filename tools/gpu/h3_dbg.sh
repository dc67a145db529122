# Phase ablation of the h3 forward kernels (timing-only: SRPDE_CONV_DBG bits make results wrong):
#   gpurun -- bash tools/gpu/h3_dbg.sh
# 1 no DMA in the loop, 2 no stage barrier, 4 no per-chunk convert, 16 no epilogue, 32 no prologue DMA,
# 64 no prologue convert, 128 no MFMAs
set -o pipefail
cd $GRAFT_REPO_ROOT
L=${1:-bridge.3,dec3.conv1,dec2.conv1,enc2.conv2,enc1.conv2,dec1.conv1}
for D in 0 16 4 20 2 23 128 247; do
  echo "== dbg $D"
  SRPDE_CONV_DBG=$D timeout -k 10 120 python tools/conv_bench.py --layers $L --only fwd --iters 10 2>&1 | grep -v amdgpu || exit 1
done
