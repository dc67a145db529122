# Phase ablation of the h3r conv (timing-only builds of the same kernel, SRPDE_CONV_DBG; results wrong):
#   gpurun -- bash tools/gpu/h3r_dbg.sh TAG
set -o pipefail
T=${1:-dbg}
R=$GRAFT_REPO_ROOT
cd $R
L=enc1.conv2,dec1.conv1,dec1.conv2,out_conv1
for d in 0 16 4 20 128 148; do
  SRPDE_CONV_DBG=$d timeout -k 10 200 python tools/conv_bench.py --iters 10 --only fwd,dgrad --layers $L > gpurun_out/h3rdbg_${T}_$d.log 2>&1 || { echo "dbg $d failed"; tail gpurun_out/h3rdbg_${T}_$d.log; exit 1; }
  echo "== DBG=$d"; grep -v amdgpu gpurun_out/h3rdbg_${T}_$d.log
done
