# Round-5 evidence batch on ONE box: SQ counters of the weight gradients (bridge.3 h3p, dec1.conv2 h3h),
# config #5 accuracy + cascade line, the world-1 RCCL rehearsal, the rocprofv3 exit-fault attribution.
#   gpurun -- bash tools/gpu/r05b.sh TAG
set -o pipefail
T=${1:-r05b}
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu/pmc_conv.sh ${T}w bridge.3,dec1.conv2 wgrad > gpurun_out/${T}_pmcw.txt 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/${T}_pmcw.txt; exit 1; }
echo "== pmc wgrad"; cat gpurun_out/${T}_pmcw.txt | head -60
echo "== accuracy"; bash tools/gpu/accuracy_cascade.sh ${T} || exit 1
echo "== rccl"; bash tools/gpu/rccl_world1.sh ${T} || exit 1
echo "== pmc exit"; bash tools/gpu/pmc_exit.sh ${T}x
