# candidate h5 build (lib/dbg/libnr.so): h5 tests on it, then layer timings and eval / train forward against the tree's
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
SRPDE_LIB=$R/superresolution_for_pdes_amd/lib/dbg/libnr.so timeout -k 10 400 python -u -m pytest tests/test_gpu_h5.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/h5nr.log 2>&1 || { echo "tests failed"; grep -v amdgpu gpurun_out/h5nr.log | tail -20; exit 1; }
tail -1 gpurun_out/h5nr.log
for rep in 1 2; do
  for V in intree nr; do
    L2=$R/superresolution_for_pdes_amd/lib/dbg/lib$V.so
    [ "$V" = intree ] && L2=$R/superresolution_for_pdes_amd/lib/libsrpde_hip.so
    echo "== $V $rep"
    SRPDE_LIB=$L2 timeout -k 10 200 python -u tools/h5_ab.py --layers --reps 1 2>&1 | grep -v amdgpu | grep "h5=1" || exit 1
    for m in eval train; do
      echo "$V $rep $m $(SRPDE_LIB=$L2 timeout -k 10 200 python tools/fwd_bench.py --mode $m 2>/dev/null | tail -1 | cut -c1-60)"
    done
  done
done
