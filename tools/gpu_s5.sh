# h3 epilogue A/B: GPU kernel / unet / schedule tests, per-layer conv bench with the LDS-staged
# 16-B stores off / on (SRPDE_H3_WIDE) and three taps per stage (SRPDE_H3_TPS=3), and the bench.
# usage: bash tools/gpu_s5.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
T=${1:-s5}
timeout -k 10 600 python -u -m pytest tests/test_gpu_schedule.py tests/test_gpu_kernels.py tests/test_gpu_unet.py tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_$T.log 2>&1 || { echo "pytest failed"; grep -v amdgpu gpurun_out/pytest_$T.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_$T.log
for cfg in "SRPDE_H3_WIDE=0" "SRPDE_H3_WIDE=1" "SRPDE_H3_TPS=3"; do
  env $cfg timeout -k 10 200 python tools/conv_bench.py --only fwd,dgrad --iters 10 > gpurun_out/convbench_${T}_$cfg.log 2>&1 || { echo "convbench failed"; tail gpurun_out/convbench_${T}_$cfg.log; exit 1; }
  echo "$cfg"; grep -v amdgpu gpurun_out/convbench_${T}_$cfg.log
done
for w in 0 1; do
  SRPDE_H3_WIDE=$w timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_${T}_wide$w.json 2> gpurun_out/bench_${T}_wide$w.err || { echo "bench failed"; tail -20 gpurun_out/bench_${T}_wide$w.err; exit 1; }
  echo "wide=$w"; python -c "import json;d=json.load(open('gpurun_out/bench_${T}_wide$w.json'));print(d['ms_per_step'],d['value'],d['roofline']['launch_ms'])"
done
echo done
