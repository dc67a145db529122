# h4 barrier-count fix check + igemm epilogue A/B on the switch test's worst gradient + the GPU suite
#   gpurun -- bash tools/gpu/r04d.sh TAG
set -o pipefail
T=${1:-r04d}
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/diag_race.py 8 > gpurun_out/race_$T.txt 2>&1 || exit 1
DIAG_CONFIGS=default timeout -k 10 120 python -u tools/diag_determinism.py 2 > gpurun_out/det_$T.txt 2>&1 || exit 1
SRPDE_LIB=$R/superresolution_for_pdes_amd/lib/dbg/libsrpde_igold.so DIAG_CONFIGS=default \
  timeout -k 10 120 python -u tools/diag_determinism.py 2 > gpurun_out/det_igold_$T.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1
rc=$?
cat gpurun_out/race_$T.txt gpurun_out/det_$T.txt gpurun_out/det_igold_$T.txt
tail -30 gpurun_out/pytest_$T.log
exit $rc
