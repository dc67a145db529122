# full GPU tests, the bench (twice), the RCCL/DataParallel path at world size 1 with the wgrad side stream
# usage: bash tools/gpu_s7.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
T=${1:-s7}
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_$T.log 2>&1 || { echo "pytest failed"; grep -v amdgpu gpurun_out/pytest_$T.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_$T.log
for k in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_${T}_$k.json 2> gpurun_out/bench_${T}_$k.err || { echo "bench failed"; tail -20 gpurun_out/bench_${T}_$k.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_${T}_$k.json'));print(d['ms_per_step'],d['value'],d['roofline']['launch_ms'],d['config']['final_loss'])"
done
timeout -k 10 300 python bench.py --no-cpu-baseline --ddp --steps 10 > gpurun_out/bench_${T}_ddp.json 2> gpurun_out/bench_${T}_ddp.err || { echo "ddp bench failed"; tail -20 gpurun_out/bench_${T}_ddp.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_${T}_ddp.json'));print('ddp', d['ms_per_step'],d['value'],d['config']['final_loss'])"
echo done
