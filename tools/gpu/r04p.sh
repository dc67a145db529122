# full GPU suite, forward timings, the bench line
#   gpurun -- bash tools/gpu/r04p.sh TAG
set -o pipefail
T=${1:-r04p}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q --timeout 180 --timeout-method thread -m gpu > gpurun_out/pytest_$T.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/pytest_$T.log | tail -2
grep -E "^FAILED" gpurun_out/pytest_$T.log | head -20
[ $rc -ge 2 ] && { grep -v amdgpu gpurun_out/pytest_$T.log | tail -30; exit 1; }
for M in eval train; do
  timeout -k 10 120 python tools/fwd_bench.py --mode $M --iters 20 2>/dev/null || exit 1
done
timeout -k 10 300 python bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || exit 1
cut -c1-300 gpurun_out/bench_$T.json
python -c "import json; d=json.load(open('gpurun_out/bench_$T.json')); print(json.dumps(d['roofline']['forward']))"
exit $rc
