# Per-kernel time of the bench step, baseline library vs the tree's build, one box:
#   gpurun -- bash tools/gpu/prof_ab.sh TAG        (stats CSVs under gpurun_out/profab_TAG_{base,new}/)
set -o pipefail
T=${1:-pab}
R=$GRAFT_REPO_ROOT
cd /tmp
export TMPDIR=/tmp
for v in base new; do
  if [ $v = base ]; then export SRPDE_LIB=$R/superresolution_for_pdes_amd/lib/ab/libsrpde_hip_base.so; else unset SRPDE_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/profab_${T}_$v -o bench -- python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/profab_${T}_$v.log 2>&1 || { echo "prof $v failed"; tail $R/gpurun_out/profab_${T}_$v.log; exit 1; }
done
cd $R
python tools/kstats_diff.py gpurun_out/profab_${T}_base gpurun_out/profab_${T}_new
