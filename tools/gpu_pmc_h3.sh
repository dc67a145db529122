# SQ counters of the h3 forward conv (bridge.3, dec1.conv1): where the wave cycles go
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-pmch3}
cd /tmp
export TMPDIR=/tmp
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA" "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/gpurun_out/$T -o p$i -- python $R/tools/conv_bench.py --layers ${2:-bridge.3} --only fwd --iters 2 > $R/gpurun_out/${T}_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $R/gpurun_out/${T}_$i.log; exit 1; }
done
cd $R
python tools/pmc_summary.py gpurun_out/$T conv_fwd_h3
echo done
