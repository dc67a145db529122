# DataParallel step: does a high-priority dgrad stream (its own HW queue) restore the overlap with the wgrad stream?
set -o pipefail
T=${1:-s19}
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python bench.py --ddp --no-cpu-baseline > gpurun_out/bench_${T}_ddp.json 2> gpurun_out/bench_${T}_ddp.err || { echo "ddp failed"; exit 1; }
SRPDE_BWD_PRIORITY=1 timeout -k 10 300 python bench.py --ddp --no-cpu-baseline > gpurun_out/bench_${T}_ddpprio.json 2> gpurun_out/bench_${T}_ddpprio.err || { echo "ddp prio failed"; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_${T}_plain.json 2> gpurun_out/bench_${T}_plain.err || { echo "plain failed"; exit 1; }
for f in ddp ddpprio plain; do echo "$f: $(python -c "import json; d=json.load(open('gpurun_out/bench_${T}_$f.json')); print(d['ms_per_step'], d['value'])")"; done
cd /tmp
export TMPDIR=/tmp
SRPDE_BWD_PRIORITY=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_${T} -o bench -- python $R/bench.py --ddp --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_${T}.log 2>&1 || { echo "prof failed"; exit 1; }
echo done
