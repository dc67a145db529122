# Round-4 check: full GPU suite (h4 bit-equality, gated decoder inputs, trajectory bar, Poisson abort),
# forward kernel summaries, the h4 phase ablation, one bench line.
#   gpurun -- bash tools/gpu/r04b.sh TAG
set -o pipefail
T=${1:-r04b}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 180 --timeout-method thread -m gpu > gpurun_out/pytest_$T.log 2>&1 || { echo "pytest failed"; grep -v amdgpu gpurun_out/pytest_$T.log | tail -40; exit 1; }
tail -1 gpurun_out/pytest_$T.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -q -s --timeout 240 --timeout-method thread -m gpu -k trajectory > gpurun_out/traj_$T.log 2>&1 || { echo "trajectory failed"; tail -20 gpurun_out/traj_$T.log; exit 1; }
grep -E "drop-in dev|BN buffers" gpurun_out/traj_$T.log
bash tools/gpu/fwd_prof.sh $T || exit 1
bash tools/gpu/h4_dbg.sh > gpurun_out/h4dbg_$T.txt 2>&1 || { echo "dbg failed"; tail -5 gpurun_out/h4dbg_$T.txt; exit 1; }
cat gpurun_out/h4dbg_$T.txt
timeout -k 10 500 python bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || { echo "bench failed"; tail -20 gpurun_out/bench_$T.err; exit 1; }
cat gpurun_out/bench_$T.json
