# h3 tile A/B: GPU kernel + schedule tests, per-layer conv bench with the 128-row two-per-CU
# tile off / on for every layer, and the train-step bench at a few SRPDE_H3_HALF thresholds.
# usage: bash tools/gpu_s4.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
T=${1:-s4}
timeout -k 10 600 python -u -m pytest tests/test_gpu_schedule.py tests/test_gpu_kernels.py tests/test_gpu_unet.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_$T.log 2>&1 || { echo "pytest failed"; grep -v amdgpu gpurun_out/pytest_$T.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_$T.log
for hv in 0 99; do
  SRPDE_H3_HALF=$hv timeout -k 10 200 python tools/conv_bench.py --only fwd,dgrad --iters 10 > gpurun_out/convbench_${T}_half$hv.log 2>&1 || { echo "convbench failed"; tail gpurun_out/convbench_${T}_half$hv.log; exit 1; }
  echo "half=$hv"; grep -v amdgpu gpurun_out/convbench_${T}_half$hv.log
done
for hv in 0 4 8; do
  SRPDE_H3_HALF=$hv timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_${T}_half$hv.json 2> gpurun_out/bench_${T}_half$hv.err || { echo "bench failed"; tail -20 gpurun_out/bench_${T}_half$hv.err; exit 1; }
  echo "half=$hv"; python -c "import json;d=json.load(open('gpurun_out/bench_${T}_half$hv.json'));print(d['ms_per_step'],d['value'])"
done
echo done
