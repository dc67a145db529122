# Round-5 side evidence on the final tree: Poisson and cascade bench lines, forward kernel summaries,
# and the per-layer conv table (the 40x40 layers as training runs them: no stored split, h3x).
#   gpurun -- bash tools/gpu/r05e.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --workload poisson > gpurun_out/r05e_bench_poisson.json 2> gpurun_out/r05e_bench_poisson.err || { echo "poisson failed"; tail -5 gpurun_out/r05e_bench_poisson.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r05e_bench_poisson.json')); print('poisson', d['value'], d['unit'])"
timeout -k 10 200 python bench.py --workload cascade > gpurun_out/r05e_bench_cascade.json 2> gpurun_out/r05e_bench_cascade.err || { echo "cascade failed"; tail -5 gpurun_out/r05e_bench_cascade.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r05e_bench_cascade.json')); print('cascade', d['value'], d['unit'], d.get('ms_per_step'))"
bash tools/gpu/fwd_prof.sh r05e > gpurun_out/fwdprof_r05e.txt 2>&1 || { echo "fwd prof failed"; tail -5 gpurun_out/fwdprof_r05e.txt; exit 1; }
bash tools/gpu/conv_table.sh r05e || exit 1
echo "r05e done"
