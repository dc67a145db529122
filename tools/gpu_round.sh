# usage: bash tools/gpu_round.sh TAG  -- tests + bench + kernel-trace profile, each step time-limited
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-x}
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_$TAG.log 2>&1; echo "pytest rc=$?"
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 10 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; exit 1; }
echo "bench ok"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1
echo "prof rc=$?"
