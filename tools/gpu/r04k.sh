# full GPU suite, SQ counters of three h4 layers (fwd, dgrad), the bench line
#   gpurun -- bash tools/gpu/r04k.sh TAG
set -o pipefail
T=${1:-r04k}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q --timeout 180 --timeout-method thread -m gpu > gpurun_out/pytest_$T.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/pytest_$T.log | tail -2
grep -E "^FAILED" gpurun_out/pytest_$T.log | head -20
[ $rc -ge 2 ] && { grep -v amdgpu gpurun_out/pytest_$T.log | tail -30; exit 1; }
bash tools/gpu/pmc_conv.sh ${T}f enc1.conv2,bridge.3,dec2.conv1 fwd > gpurun_out/pmc_${T}_fwd.txt 2>&1 || { tail -5 gpurun_out/pmc_${T}_fwd.txt; exit 1; }
bash tools/gpu/pmc_conv.sh ${T}d enc1.conv2,bridge.3,dec2.conv1 dgrad > gpurun_out/pmc_${T}_dgrad.txt 2>&1 || { tail -5 gpurun_out/pmc_${T}_dgrad.txt; exit 1; }
grep -E "^\(|WAIT_ANY /|VALU/MFMA" gpurun_out/pmc_${T}_fwd.txt gpurun_out/pmc_${T}_dgrad.txt
timeout -k 10 300 python bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || exit 1
cut -c1-400 gpurun_out/bench_$T.json
exit $rc
