# Train-step A/B of an environment switch on ONE box, interleaved:  gpurun -- bash tools/gpu/env_ab.sh TAG REPS VAR=VALUE...
set -o pipefail
T=$1; N=$2; shift 2
R=$GRAFT_REPO_ROOT
cd $R
for rep in $(seq 1 $N); do
  for v in base new; do
    if [ $v = new ]; then
      env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --no-live-traffic --steps 20 > gpurun_out/envab_${T}_${v}_$rep.json 2> gpurun_out/envab_${T}_${v}_$rep.err || { tail -5 gpurun_out/envab_${T}_${v}_$rep.err; exit 1; }
    else
      timeout -k 10 200 python bench.py --no-cpu-baseline --no-live-traffic --steps 20 > gpurun_out/envab_${T}_${v}_$rep.json 2> gpurun_out/envab_${T}_${v}_$rep.err || { tail -5 gpurun_out/envab_${T}_${v}_$rep.err; exit 1; }
    fi
    echo "$v $rep $(python -c "import json; d=json.load(open('gpurun_out/envab_${T}_${v}_$rep.json')); print(d['ms_per_step'])")"
  done
done
