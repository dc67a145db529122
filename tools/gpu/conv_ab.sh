# Conv kernel change check on ONE box: kernel parity tests on the new build, then per-layer timing
# of the baseline build (lib/dbg/libsrpde_base.so, SRPDE_LIB) and the new one, interleaved twice.
#   gpurun -- bash tools/gpu/conv_ab.sh TAG [LAYERS] [PASSES]
set -o pipefail
T=${1:-ab}
L=${2:-}
K=${3:-fwd,dgrad}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_h4.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu -k "conv or h3 or h4" > gpurun_out/ab_pytest_$T.log 2>&1 || { echo "tests failed"; grep -v amdgpu gpurun_out/ab_pytest_$T.log | tail -20; exit 1; }
tail -1 gpurun_out/ab_pytest_$T.log
LA=""
[ -n "$L" ] && LA="--layers $L"
for rep in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export SRPDE_LIB=$R/superresolution_for_pdes_amd/lib/dbg/libsrpde_base.so; else unset SRPDE_LIB; fi
    timeout -k 10 300 python tools/conv_bench.py --iters 10 --only $K $LA --json-out gpurun_out/ab_${T}_${v}_$rep.json > gpurun_out/ab_${T}_${v}_$rep.log 2>&1 || { echo "bench $v failed"; tail gpurun_out/ab_${T}_${v}_$rep.log; exit 1; }
  done
done
unset SRPDE_LIB
python tools/ab_compare.py gpurun_out/ab_${T}
