# The rocprofv3 --pmc exit fault after a cooperative launch (verdict r4 #6): the failing pass again with this
# process's memory map saved at Python exit (bench.py SRPDE_DUMP_MAPS), the crash frames attributed to the
# mapped objects, then the same pass over each case alone.   gpurun -- bash tools/gpu/pmc_exit.sh TAG
set -o pipefail
T=${1:-pmcx}
R=$GRAFT_REPO_ROOT
cd /tmp
export TMPDIR=/tmp
i=0
for S in "80:1024,640:4" "640:4" "80:1024"; do
  i=$((i+1))
  SRPDE_DUMP_MAPS=$R/gpurun_out/${T}_maps_$i.txt timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/${T}_$i -o p -- python $R/bench.py --workload poisson --poisson-sizes $S --steps 2 --warmup 1 --no-cpu-baseline --no-live-traffic > $R/gpurun_out/${T}_$i.log 2>&1
  echo "pass $i ($S): exit $?"
  python $R/tools/attribute_frames.py $R/gpurun_out/${T}_$i.log $R/gpurun_out/${T}_maps_$i.txt 2>&1 | head -30
done
exit 0
