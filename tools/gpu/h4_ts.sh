# phase timestamps of the h4 kernel (timestamp build) for a few layers
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export SRPDE_LIB=$R/superresolution_for_pdes_amd/lib/dbg/libsrpde_dbg256.so
for L in enc1.conv2 dec1.conv1 enc2.conv2 bridge.3; do
  timeout -k 10 60 python tools/h4_phase_ts.py $L 2>&1 | grep -v amdgpu || exit 1
done
