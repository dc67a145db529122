# SQ counters of selected conv layers / passes:  gpurun -- bash tools/gpu/pmc_conv.sh TAG LAYERS PASS
set -o pipefail
T=${1:-pmc}
L=${2:-enc1.conv2,bridge.3}
K=${3:-fwd}
R=$GRAFT_REPO_ROOT
cd /tmp
export TMPDIR=/tmp
i=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/gpurun_out/pmcc_$T -o p$i -- python $R/tools/conv_bench.py --layers $L --only $K --iters 2 > $R/gpurun_out/pmcc_${T}_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $R/gpurun_out/pmcc_${T}_$i.log; exit 1; }
done
cd $R
python tools/pmc_by_grid.py gpurun_out/pmcc_$T
