# The full GPU suite, smoke(), then the bench line (no CPU baseline / live traffic): a quick whole-tree check.
#   gpurun -- bash tools/gpu/tests_bench.sh TAG
set -o pipefail
T=${1:-tb}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/tb_pytest_$T.log 2>&1 || { echo "pytest failed"; grep -v amdgpu gpurun_out/tb_pytest_$T.log | tail -40; exit 1; }
tail -1 gpurun_out/tb_pytest_$T.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/tb_smoke_$T.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/tb_smoke_$T.log; exit 1; }
tail -1 gpurun_out/tb_smoke_$T.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-live-traffic > gpurun_out/tb_bench_$T.json 2> gpurun_out/tb_bench_$T.err || { echo "bench failed"; tail -20 gpurun_out/tb_bench_$T.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/tb_bench_$T.json')); print(d['ms_per_step'], d['value'], d['roofline']['forward']['eval']['ms'], d['roofline']['forward']['train']['ms'])"
