# forward kernel summaries (eval / train) + the h4 phase ablation on the W = 40 layers and bridge.3
#   gpurun -- bash tools/gpu/r04g.sh TAG
set -o pipefail
T=${1:-r04g}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu/fwd_prof.sh $T || exit 1
bash tools/gpu/h4_dbg.sh enc1.conv2,dec1.conv1,dec1.conv2,bridge.3,enc2.conv2 > gpurun_out/h4dbg_$T.txt 2>&1 || { tail -5 gpurun_out/h4dbg_$T.txt; exit 1; }
cat gpurun_out/h4dbg_$T.txt
