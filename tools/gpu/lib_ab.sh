# Per-layer conv A/B of the baseline library (tools/build_base.sh) against the tree's build, interleaved;
# optional pytest -k selector run on the new build first.
#   gpurun -- bash tools/gpu/lib_ab.sh [LAYERS] [PASSES] [PYTEST_K]
set -o pipefail
cd $GRAFT_REPO_ROOT
L=${1:-enc2.conv2,enc3.conv2,bridge.0,bridge.3,dec3.conv1,dec2.conv1}
O=${2:-fwd,dgrad}
if [ -n "$3" ]; then
  timeout -k 10 300 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "$3" > gpurun_out/libab_pytest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/libab_pytest.log; exit 1; }
  tail -1 gpurun_out/libab_pytest.log
fi
for rep in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export SRPDE_LIB=$GRAFT_REPO_ROOT/superresolution_for_pdes_amd/lib/ab/libsrpde_hip_base.so; else unset SRPDE_LIB; fi
    echo "== $v $rep"
    timeout -k 10 120 python tools/conv_bench.py --layers $L --only $O --iters 10 2>&1 | grep -v amdgpu || exit 1
  done
done
