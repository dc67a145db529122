# A/B of the 4-wave (one per SIMD) 256x128 h3 layout against the 8-wave one, per layer
set -o pipefail
cd $GRAFT_REPO_ROOT
L=${1:-enc2.conv2,enc3.conv2,bridge.0,bridge.3,dec3.conv1,dec2.conv1}
for W in 0 1 0 1; do
  echo "== SRPDE_H3_W4=$W"
  SRPDE_H3_W4=$W timeout -k 10 120 python tools/conv_bench.py --layers $L --only fwd,dgrad --iters 10 2>&1 | grep -v amdgpu || exit 1
done
