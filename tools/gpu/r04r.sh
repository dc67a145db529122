# round-4 evidence: round_evidence.sh (GPU tests, smoke, PMC traffic, bench, rocprof stats), forward timings,
# the Poisson and cascade lines
#   gpurun -- bash tools/gpu/r04r.sh TAG
set -o pipefail
T=${1:-r04r}
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
bash tools/gpu/round_evidence.sh $T || exit 1
cd $R
for M in eval train; do
  timeout -k 10 120 python tools/fwd_bench.py --mode $M --iters 20 2>/dev/null | tee gpurun_out/fwd_${M}_$T.txt || exit 1
done
timeout -k 10 400 python bench.py --workload poisson > gpurun_out/bench_poisson_$T.json 2> gpurun_out/bench_poisson_$T.err || { echo "poisson bench failed"; exit 1; }
cut -c1-400 gpurun_out/bench_poisson_$T.json
python -c "import sys, torch; sys.path.insert(0, 'tests/golden'); from state import fixture_state_torch; torch.save(fixture_state_torch(), 'gpurun_out/cascade20_state.pt')" || exit 1
timeout -k 10 400 python bench.py --workload cascade --checkpoint gpurun_out/cascade20_state.pt \
  --cascade-fixture tests/golden/cascade640_fixture.npz --steps 10 --warmup 2 > gpurun_out/bench_cascade_$T.json 2> gpurun_out/bench_cascade_$T.err || { echo "cascade bench failed"; exit 1; }
cut -c1-300 gpurun_out/bench_cascade_$T.json
