# DMA-placement variants of the 8-wave h3 kernel (SRPDE_CONV_DBG 256 / 512: exact results), per layer
set -o pipefail
cd $GRAFT_REPO_ROOT
L=${1:-enc2.conv2,bridge.0,bridge.3,dec3.conv1,dec2.conv1}
for D in 0 256 512 0 256 512; do
  echo "== dbg $D"
  SRPDE_CONV_DBG=$D timeout -k 10 120 python tools/conv_bench.py --layers $L --only fwd,dgrad --iters 10 2>&1 | grep -v amdgpu | grep TOTAL || exit 1
done
SRPDE_CONV_DBG=512 timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu -k "conv" > gpurun_out/dma_pytest.log 2>&1; tail -1 gpurun_out/dma_pytest.log
