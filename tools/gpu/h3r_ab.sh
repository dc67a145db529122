# h3r (register-staged 4-wave conv, two workgroups per CU) against the 8-wave kernel on ONE box:
# equality + conv tests, per-layer timing of the shallow-K layers, and the train step, each knob.
#   gpurun -- bash tools/gpu/h3r_ab.sh TAG
set -o pipefail
T=${1:-h3r}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_schedule.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu -k "conv or h3" > gpurun_out/h3r_pytest_$T.log 2>&1 || { echo "tests failed"; grep -v amdgpu gpurun_out/h3r_pytest_$T.log | tail -30; exit 1; }
tail -1 gpurun_out/h3r_pytest_$T.log
L=enc1.conv2,enc2.conv1,dec1.conv1,dec1.conv2,out_conv1,out_conv2
for rep in 1 2; do
  for v in 0 1; do
    if [ $v = e ]; then export SRPDE_H3R=1 SRPDE_H3R_EARLY=1; else export SRPDE_H3R=$v SRPDE_H3R_EARLY=0; fi
    timeout -k 10 200 python tools/conv_bench.py --iters 10 --only fwd,dgrad --layers $L > gpurun_out/h3r_conv_${T}_${v}_$rep.log 2>&1 || { echo "conv bench $v failed"; tail gpurun_out/h3r_conv_${T}_${v}_$rep.log; exit 1; }
    echo "== H3R=$v rep $rep"; cat gpurun_out/h3r_conv_${T}_${v}_$rep.log
  done
done
for v in 0 1 0 1; do
  if [ $v = e ]; then export SRPDE_H3R=1 SRPDE_H3R_EARLY=1; else export SRPDE_H3R=$v SRPDE_H3R_EARLY=0; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-live-traffic --steps 20 > gpurun_out/h3r_bench_${T}_$v.json 2> gpurun_out/h3r_bench_${T}_$v.err || { echo "bench $v failed"; tail gpurun_out/h3r_bench_${T}_$v.err; exit 1; }
  echo "H3R=$v $(python -c "import json,sys; d=json.load(open('gpurun_out/h3r_bench_${T}_$v.json')); print(d['ms_per_step'], d['value'])")"
done
