# SQ counters of the h5 forward (one layer, eval + train variants) and the same-process A/B of diagnostic
# builds:  gpurun -- bash tools/gpu/h5_pmc.sh TAG [LAYER] [LIBS...]   (LIBS: lib/dbg/*.so variants)
set -o pipefail
T=${1:-h5p}
L=${2:-enc1.conv2}
shift 2
R=$GRAFT_REPO_ROOT
cd /tmp
export TMPDIR=/tmp
i=0
for M in eval train; do
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/gpurun_out/pmch5_$T -o p${M}$i -- python $R/tools/h5_one.py --layer $L --mode $M --iters 3 > $R/gpurun_out/pmch5_${T}_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $R/gpurun_out/pmch5_${T}_$i.log; exit 1; }
done
done
cd $R
python tools/pmc_by_grid.py gpurun_out/pmch5_$T 2>&1 | tee gpurun_out/pmch5_$T.txt
for LIB in "$@"; do
  echo "== $LIB"
  SRPDE_LIB=$R/$LIB timeout -k 10 200 python -u tools/h5_ab.py --layers --reps 1 2>&1 | grep -v amdgpu | grep "h5=1"
done
