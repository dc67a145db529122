# full GPU tests + bench (side stream on/off) + rocprof kernel trace of the bench
# usage: bash tools/gpu_s8.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
T=${1:-s8}
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_$T.log 2>&1 || { echo "pytest failed"; grep -v amdgpu gpurun_out/pytest_$T.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_$T.log
for ws in 1 0 1; do
  SRPDE_WGRAD_STREAM=$ws timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_${T}_ws$ws.json 2> gpurun_out/bench_${T}_ws$ws.err || { echo "bench failed"; tail -20 gpurun_out/bench_${T}_ws$ws.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_${T}_ws$ws.json'));print('ws=$ws',d['ms_per_step'],d['value'],d['roofline']['launch_ms'],d['config']['final_loss'])"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$T -o bench -- python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_$T.log 2>&1 || { echo "prof failed"; exit 1; }
echo done
