# SQ counters of the Poisson CG kernels (LDS CG at n=80, grid CG at 640):  gpurun -- bash tools/gpu/pmc_poisson.sh TAG
set -o pipefail
T=${1:-pmcp}
R=$GRAFT_REPO_ROOT
cd /tmp
export TMPDIR=/tmp
i=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/gpurun_out/pmcp_$T -o p$i -- python $R/bench.py --workload poisson --poisson-sizes 80:1024 --steps 2 --no-cpu-baseline --no-live-traffic > $R/gpurun_out/pmcp_${T}_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $R/gpurun_out/pmcp_${T}_$i.log; exit 1; }
done
cd $R
python tools/pmc_by_grid.py gpurun_out/pmcp_$T "cg_lds" | tee gpurun_out/pmcp_$T.txt
