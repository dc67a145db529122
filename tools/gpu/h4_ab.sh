# h4 check on ONE box: bit-equality tests h4 vs h3, then per-layer timing SRPDE_H4=0 (h3 8-wave) vs 1
# (h4), interleaved twice, same library.
#   gpurun -- bash tools/gpu/h4_ab.sh TAG [PASSES]
set -o pipefail
T=${1:-h4}
K=${2:-fwd,dgrad}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_h4.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/h4_pytest_$T.log 2>&1 || { echo "h4 tests failed"; grep -v amdgpu gpurun_out/h4_pytest_$T.log | tail -30; exit 1; }
tail -1 gpurun_out/h4_pytest_$T.log
L=enc2.conv1,enc2.conv2,enc3.conv1,enc3.conv2,bridge.0,bridge.3,dec3.conv1,dec3.conv2,dec2.conv1,dec2.conv2
for rep in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export SRPDE_H4=0; else export SRPDE_H4=1; fi
    timeout -k 10 300 python tools/conv_bench.py --iters 10 --only $K --layers $L --json-out gpurun_out/ab_${T}_${v}_$rep.json > gpurun_out/ab_${T}_${v}_$rep.log 2>&1 || { echo "bench $v failed"; tail gpurun_out/ab_${T}_${v}_$rep.log; exit 1; }
  done
done
unset SRPDE_H4
python tools/ab_compare.py gpurun_out/ab_${T} | tee gpurun_out/ab_${T}.txt
