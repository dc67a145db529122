# Same-box timing of several builds of the library (names under lib/dbg/libsrpde_<name>.so, "new" = the
# in-tree build), interleaved twice, per layer and pass.
#   gpurun -- bash tools/gpu/multi_ab.sh TAG "base early_prio new" [LAYERS] [PASSES]
set -o pipefail
T=${1:-mab}
V=${2:-"base new"}
L=${3:-enc1.conv2,dec1.conv1,enc2.conv2,bridge.3,dec3.conv1,dec2.conv1}
K=${4:-fwd,dgrad}
R=$GRAFT_REPO_ROOT
cd $R
for rep in 1 2; do
  for v in $V; do
    if [ $v = new ]; then unset SRPDE_LIB; else export SRPDE_LIB=$R/superresolution_for_pdes_amd/lib/dbg/libsrpde_$v.so; fi
    timeout -k 10 200 python tools/conv_bench.py --iters 10 --only $K --layers $L --json-out gpurun_out/mab_${T}_${v}_$rep.json > gpurun_out/mab_${T}_${v}_$rep.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/mab_${T}_${v}_$rep.log; exit 1; }
    echo "$v $rep $(grep TOTAL gpurun_out/mab_${T}_${v}_$rep.log | tr '\n' ' ')"
  done
done
unset SRPDE_LIB
