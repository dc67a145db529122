# Same-box bench A/B over environment knobs:  gpurun -- bash tools/gpu/bench_knobs.sh TAG "VAR=a VAR=b ..."
set -o pipefail
T=${1:-knob}
R=$GRAFT_REPO_ROOT
cd $R
for rep in 1 2; do
  for kv in $2; do
    timeout -k 10 200 env $kv python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-traffic > gpurun_out/knob_${T}_${kv}_$rep.json 2> gpurun_out/knob_${T}_${kv}_$rep.err || { echo "bench $kv failed"; tail -5 gpurun_out/knob_${T}_${kv}_$rep.err; exit 1; }
    python -c "import json,sys; r=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], r['ms_per_step'], r['roofline']['launch_ms'])" gpurun_out/knob_${T}_${kv}_$rep.json $kv $rep
  done
done
