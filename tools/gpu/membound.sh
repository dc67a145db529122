# HBM-bound backward kernels of one B = 1024 training step, in the step and alone (tools/membound_table.py):
# a kernel trace and two PMC passes (FETCH_SIZE, WRITE_SIZE), each its own run.
#   gpurun -- bash tools/gpu/membound.sh TAG      -> gpurun_out/membound_TAG.md
set -o pipefail
T=${1:-mb}
R=$GRAFT_REPO_ROOT
cd /tmp
export TMPDIR=/tmp
O=$R/gpurun_out/membound_$T
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o t -- python3 $R/tools/membound_table.py run $O/calls.json > $O/trace.log 2>&1 || { echo "trace pass failed"; tail -20 $O/trace.log; exit 1; }
i=0
for C in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $C --output-format csv -d $O/pmc$i -o p -- python3 $R/tools/membound_table.py run $O/calls_pmc$i.json > $O/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -20 $O/pmc$i.log; exit 1; }
done
cd $R
python3 tools/membound_table.py table $O/calls.json $O/trace $O/pmc1 $O/pmc2 > gpurun_out/membound_$T.md && cat gpurun_out/membound_$T.md | tail -25
