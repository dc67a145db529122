# n16 / head launch bounds / h4 convert unroll: tests on the tree's build, then forward (eval, train) and
# train-step timings of lib/dbg/lib{head,up1,up2}.so and the tree's build, interleaved on one box
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_h5.py tests/test_gpu_unet.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r05c_pytest.log 2>&1 || { echo "tests failed"; grep -v amdgpu gpurun_out/r05c_pytest.log | tail -25; exit 1; }
tail -1 gpurun_out/r05c_pytest.log
SRPDE_LIB=$R/superresolution_for_pdes_amd/lib/dbg/libup2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_h4.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r05c_pytest_up2.log 2>&1 || { echo "up2 tests failed"; tail -20 gpurun_out/r05c_pytest_up2.log; exit 1; }
tail -1 gpurun_out/r05c_pytest_up2.log
for rep in 1 2; do
  for V in head intree up1 up2; do
    L2=$R/superresolution_for_pdes_amd/lib/dbg/lib$V.so
    [ "$V" = intree ] && L2=$R/superresolution_for_pdes_amd/lib/libsrpde_hip.so
    e=$(SRPDE_LIB=$L2 timeout -k 10 200 python tools/fwd_bench.py --mode eval 2>/dev/null | tail -1 | python -c "import json,sys; print(json.load(sys.stdin)['ms'])")
    t=$(SRPDE_LIB=$L2 timeout -k 10 200 python tools/fwd_bench.py --mode train 2>/dev/null | tail -1 | python -c "import json,sys; print(json.load(sys.stdin)['ms'])")
    s=$(SRPDE_LIB=$L2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-live-traffic --steps 20 2>/dev/null | python -c "import json,sys; print(json.load(sys.stdin)['ms_per_step'])")
    echo "$V $rep eval $e train $t step $s"
  done
done
