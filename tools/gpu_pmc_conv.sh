# PMC passes (each its own rocprofv3 run, counters only + kernel trace) over the conv micro-bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
L=${1:-bridge.3}
K=${2:-fwd}
i=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
         "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/gpurun_out/pmc_${L}_${K} -o p$i -- python $R/tools/conv_bench.py --layers $L --only $K --iters 3 ${3:+--math $3} > $R/gpurun_out/pmc_${L}_${K}_$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo pmc done
