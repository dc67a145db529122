# h4 tail fused into the conv kernel: h4 / kernel tests, then eval / train forward timings and the bench,
# against the build before it (same box)
#   gpurun -- bash tools/gpu/tailfuse.sh TAG
set -o pipefail
T=${1:-tf}
OLD=superresolution_for_pdes_amd/lib/dbg/libsrpde_notailfuse.so
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_h4.py tests/test_gpu_kernels.py -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/tf_tests_$T.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/tf_tests_$T.log | tail -1
grep -E "^FAILED" gpurun_out/tf_tests_$T.log | head -20
[ $rc -ge 2 ] && { grep -v amdgpu gpurun_out/tf_tests_$T.log | tail -30; exit 1; }
for L in old new old new; do
  if [ $L = old ]; then export SRPDE_LIB=$OLD; else unset SRPDE_LIB; fi
  for M in eval train; do
    echo -n "$L "; timeout -k 10 120 python tools/fwd_bench.py --mode $M --iters 20 2>/dev/null || exit 1
  done
done
exit $rc
