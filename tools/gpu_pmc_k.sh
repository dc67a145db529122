# SQ / TCC counters of one conv kernel family on one layer:  bash tools/gpu_pmc_k.sh TAG LAYER ONLY PATTERN
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-pmck}; L=${2:-bridge.3}; O=${3:-wgrad}; PAT=${4:-conv_wgrad_h3p}
cd /tmp
export TMPDIR=/tmp
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/gpurun_out/$T -o p$i -- python $R/tools/conv_bench.py --layers $L --only $O --iters 2 > $R/gpurun_out/${T}_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $R/gpurun_out/${T}_$i.log; exit 1; }
done
cd $R
python tools/pmc_summary.py gpurun_out/$T $PAT

echo done
