# HBM traffic (FETCH_SIZE, WRITE_SIZE: one pass each) of the pointwise kernels at the step's shapes.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp
export TMPDIR=/tmp
i=0
for C in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/gpurun_out/pmc_pw -o p$i -- python $R/tools/pw_bench.py --iters 2 > $R/gpurun_out/pmc_pw_$i.log 2>&1 || { echo "pmc pass $i failed"; tail $R/gpurun_out/pmc_pw_$i.log; exit 1; }
done
echo done
