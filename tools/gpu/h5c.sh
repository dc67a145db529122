# h5 tests + A/B + per-tap timestamps (lib/dbg/libh5ts.so) + no-MFMA variant:  gpurun -- bash tools/gpu/h5c.sh TAG
set -o pipefail
T=${1:-h5}
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu/h5.sh $T || exit $?
if [ -f superresolution_for_pdes_amd/lib/dbg/libh5dbg2.so ]; then
  echo "== no MFMA"
  SRPDE_LIB=$R/superresolution_for_pdes_amd/lib/dbg/libh5dbg2.so timeout -k 10 200 python -u tools/h5_ab.py --layers --reps 1 2>&1 | grep -v amdgpu | grep "h5=1" || exit 1
fi
if [ -f superresolution_for_pdes_amd/lib/dbg/libh5ts.so ]; then
  SRPDE_LIB=$R/superresolution_for_pdes_amd/lib/dbg/libh5ts.so timeout -k 10 120 python tools/h5_phase_ts.py enc1.conv2 eval 2>&1 | grep -v amdgpu || exit 1
fi
