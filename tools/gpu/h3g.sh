# h3g (deep weight gradient, input-row ring) on one box: its tests, the weight-gradient tests around it, then a
# same-box A/B against lib/dbg/libsrpde_base.so (built with -DSRPDE_NO_H3G): per-layer wgrad timing and the step.
#   gpurun -- bash tools/gpu/h3g.sh TAG
set -o pipefail
T=${1:-g}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_wgrad_g.py tests/test_gpu_wgrad_x.py tests/test_gpu_b1024.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/h3g_pytest_$T.log 2>&1 || { echo "tests failed"; grep -v amdgpu gpurun_out/h3g_pytest_$T.log | tail -30; exit 1; }
tail -1 gpurun_out/h3g_pytest_$T.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu -k "wgrad or split" > gpurun_out/h3g_pytest2_$T.log 2>&1 || { echo "kernel tests failed"; grep -v amdgpu gpurun_out/h3g_pytest2_$T.log | tail -30; exit 1; }
tail -1 gpurun_out/h3g_pytest2_$T.log
LAY=enc2.conv1,enc2.conv2,enc3.conv1,enc3.conv2,bridge.0,bridge.3,dec3.conv1,dec3.conv2,dec2.conv1,dec2.conv2
for rep in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export SRPDE_LIB=$R/superresolution_for_pdes_amd/lib/dbg/libsrpde_base.so; else unset SRPDE_LIB; fi
    timeout -k 10 300 python tools/conv_bench.py --iters 10 --only wgrad --layers $LAY --json-out gpurun_out/ab_${T}_${v}_$rep.json > gpurun_out/ab_${T}_${v}_$rep.log 2>&1 || { echo "bench $v failed"; tail gpurun_out/ab_${T}_${v}_$rep.log; exit 1; }
  done
done
unset SRPDE_LIB
python tools/ab_compare.py gpurun_out/ab_${T}
for rep in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export SRPDE_LIB=$R/superresolution_for_pdes_amd/lib/dbg/libsrpde_base.so; else unset SRPDE_LIB; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-live-traffic --steps 20 --warmup 3 > gpurun_out/step_${T}_${v}_$rep.json 2> gpurun_out/step_${T}_${v}_$rep.err || { echo "step $v failed"; tail gpurun_out/step_${T}_${v}_$rep.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/step_${T}_${v}_$rep.json')); print('$v', d['ms_per_step'], d['roofline']['kernels'][0]['kernel'], d['roofline']['kernels'][0]['frac'])"
  done
done
