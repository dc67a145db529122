# h4 tap barrier after every second tap (-DH4_BAR2=1, lib/dbg/libsrpde_bar2.so) against the default build
# (lib/dbg/libsrpde_base.so): parity tests and the run-to-run race check on the variant, then per-layer
# conv timing and the eval / train forward, alternating on one box
#   gpurun -- bash tools/gpu/bar2_ab.sh TAG
set -o pipefail
T=${1:-bar2}
R=$GRAFT_REPO_ROOT
B=$R/superresolution_for_pdes_amd/lib/dbg/libsrpde_base.so
V=$R/superresolution_for_pdes_amd/lib/dbg/libsrpde_bar2.so
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
export SRPDE_LIB=$V
timeout -k 10 400 python -u -m pytest tests/test_gpu_h4.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/bar2_pytest_$T.log 2>&1 || { echo "tests failed"; grep -v amdgpu gpurun_out/bar2_pytest_$T.log | tail -20; exit 1; }
tail -1 gpurun_out/bar2_pytest_$T.log
timeout -k 10 300 python -u tools/diag_race.py 6 > gpurun_out/bar2_race_$T.log 2>&1 || { echo "race diag failed"; tail -20 gpurun_out/bar2_race_$T.log; exit 1; }
tail -8 gpurun_out/bar2_race_$T.log
for rep in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export SRPDE_LIB=$B; else export SRPDE_LIB=$V; fi
    timeout -k 10 300 python tools/conv_bench.py --iters 10 --only fwd,dgrad --json-out gpurun_out/bar2_${T}_${v}_$rep.json > gpurun_out/bar2_${T}_${v}_$rep.log 2>&1 || { echo "bench $v failed"; tail gpurun_out/bar2_${T}_${v}_$rep.log; exit 1; }
    for M in eval train; do
      echo -n "$v "; timeout -k 10 120 python tools/fwd_bench.py --mode $M --iters 20 2>/dev/null || exit 1
    done
  done
done
python tools/ab_compare.py gpurun_out/bar2_${T}
