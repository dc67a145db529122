# Round-4 check (continues past test FAILURES, stops at crashes / timeouts): cascade bisect, full GPU
# suite, trajectory numbers, forward kernel summaries, h4 phase ablation, one bench line.
#   gpurun -- bash tools/gpu/r04c.sh TAG
set -o pipefail
T=${1:-r04c}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/diag_cascade20.py > gpurun_out/cascade20_$T.txt 2>&1; rc=$?
grep -v amdgpu gpurun_out/cascade20_$T.txt | tail -12
[ $rc -ne 0 ] && { echo "cascade diag rc=$rc"; [ $rc -ge 124 ] && exit 1; }
timeout -k 10 900 python -u -m pytest tests -q --timeout 180 --timeout-method thread -m gpu > gpurun_out/pytest_$T.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/pytest_$T.log | tail -3
grep -E "^FAILED" gpurun_out/pytest_$T.log | head -20
[ $rc -ge 2 ] && { echo "pytest rc=$rc"; grep -v amdgpu gpurun_out/pytest_$T.log | tail -30; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -q -s --timeout 240 --timeout-method thread -m gpu -k trajectory > gpurun_out/traj_$T.log 2>&1
grep -E "drop-in dev|BN buffers|passed|failed" gpurun_out/traj_$T.log
bash tools/gpu/fwd_prof.sh $T || exit 1
bash tools/gpu/h4_dbg.sh > gpurun_out/h4dbg_$T.txt 2>&1 || { echo "dbg failed"; tail -5 gpurun_out/h4dbg_$T.txt; exit 1; }
cat gpurun_out/h4dbg_$T.txt
timeout -k 10 500 python bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || { echo "bench failed"; tail -20 gpurun_out/bench_$T.err; exit 1; }
cat gpurun_out/bench_$T.json
