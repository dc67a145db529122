# h4 convert-loop unroll A/B: h4 tests on the candidate, layer timings, eval/train forward  (gpurun -- bash tools/gpu/h4u.sh)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
SRPDE_LIB=$R/superresolution_for_pdes_amd/lib/dbg/libup2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_h4.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/h4u.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/h4u.log; exit 1; }
tail -1 gpurun_out/h4u.log
bash tools/gpu/h4_variants.sh u bridge.3,dec3.conv1,enc2.conv2,dec2.conv2,enc1.conv2 fwd,dgrad up2 up1 || exit 1
for rep in 1 2; do
  for V in intree up1 up2; do
    L2=$R/superresolution_for_pdes_amd/lib/dbg/lib$V.so
    [ "$V" = intree ] && L2=$R/superresolution_for_pdes_amd/lib/libsrpde_hip.so
    for m in eval train; do
      echo "$V $rep $m $(SRPDE_LIB=$L2 timeout -k 10 200 python tools/fwd_bench.py --mode $m 2>/dev/null | tail -1 | cut -c1-80)"
    done
  done
done
