# h5 tests + layer times of candidate builds (lib/dbg/lib<NAME>.so):  gpurun -- bash tools/gpu/h5_libs.sh TAG NAME...
set -o pipefail
T=$1; shift
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
for V in "$@"; do
  echo "== $V"
  SRPDE_LIB=$R/superresolution_for_pdes_amd/lib/dbg/lib$V.so timeout -k 10 300 python -u -m pytest tests/test_gpu_h5.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/h5libs_${T}_$V.log 2>&1 || { echo "tests failed"; grep -v amdgpu gpurun_out/h5libs_${T}_$V.log | tail -20; exit 1; }
  tail -1 gpurun_out/h5libs_${T}_$V.log
  SRPDE_LIB=$R/superresolution_for_pdes_amd/lib/dbg/lib$V.so timeout -k 10 200 python -u tools/h5_ab.py --layers --reps 1 2>&1 | grep -v amdgpu | grep "h5=1" || exit 1
done
