# Round-end evidence on one MI355X: full GPU tests, smoke, HBM-traffic PMC passes for the
# roofline kernel (bridge.3 forward conv) kept as profiles/traffic_*.json, the bench line exactly as
# the driver runs it (which measures the same traffic live), and the kernel-trace stats of the bench
# command.
# usage: bash tools/gpu_round.sh TAG     (outputs under gpurun_out/, copy what is judged to profiles/)
set -o pipefail
T=${1:-final}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_$T.log 2>&1 || { echo "pytest failed"; grep -v amdgpu gpurun_out/pytest_$T.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_$T.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_$T.log; exit 1; }
tail -1 gpurun_out/smoke_$T.log
cd /tmp
i=0
for C in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/gpurun_out/pmc_$T -o p$i -- python $R/tools/conv_bench.py --layers bridge.3 --only fwd --iters 3 > $R/gpurun_out/pmc_${T}_$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
cd $R
python tools/traffic_json.py gpurun_out/pmc_$T bridge.3 gpurun_out/traffic_$T.json
timeout -k 10 500 python bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || { echo "bench failed"; tail -20 gpurun_out/bench_$T.err; exit 1; }
cat gpurun_out/bench_$T.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$T -o bench -- python $R/bench.py --no-cpu-baseline --no-live-traffic > $R/gpurun_out/prof_$T.log 2>&1 || { echo "prof failed"; exit 1; }
echo "round evidence done"
