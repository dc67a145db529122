# persistent h3 tile walk A/B: schedule + kernel tests, per-layer conv bench with
# SRPDE_H3_PERSIST=0 / 1, and the bench at both.   usage: bash tools/gpu_s6.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
T=${1:-s6}
timeout -k 10 600 python -u -m pytest tests/test_gpu_schedule.py tests/test_gpu_kernels.py tests/test_gpu_unet.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_$T.log 2>&1 || { echo "pytest failed"; grep -v amdgpu gpurun_out/pytest_$T.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_$T.log
for pm in 0 1; do
  SRPDE_H3_PERSIST=$pm timeout -k 10 200 python tools/conv_bench.py --only fwd,dgrad --iters 10 > gpurun_out/convbench_${T}_p$pm.log 2>&1 || { echo "convbench failed"; tail gpurun_out/convbench_${T}_p$pm.log; exit 1; }
  echo "persist=$pm"; grep -v amdgpu gpurun_out/convbench_${T}_p$pm.log
done
for pm in 0 1; do
  SRPDE_H3_PERSIST=$pm timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_${T}_p$pm.json 2> gpurun_out/bench_${T}_p$pm.err || { echo "bench failed"; tail -20 gpurun_out/bench_${T}_p$pm.err; exit 1; }
  echo "persist=$pm"; python -c "import json;d=json.load(open('gpurun_out/bench_${T}_p$pm.json'));print(d['ms_per_step'],d['value'],d['roofline']['launch_ms'])"
done
echo done
