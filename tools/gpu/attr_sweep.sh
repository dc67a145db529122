# Same-box sweep of one executor attribute (tools/bench_with.py) over several values, alternating, REPS rounds.
#   gpurun -- bash tools/gpu/attr_sweep.sh TAG module.ATTR "v1 v2 ..." [REPS]
set -o pipefail
T=$1; ATTR=$2; VALS=$3; N=${4:-2}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
for rep in $(seq 1 $N); do
  for v in $VALS; do
    timeout -k 10 200 python tools/bench_with.py $ATTR=$v -- --no-cpu-baseline --no-live-traffic --steps 20 --warmup 3 > gpurun_out/sw_${T}_${v}_$rep.json 2> gpurun_out/sw_${T}_${v}_$rep.err || { echo "bench $v failed"; tail gpurun_out/sw_${T}_${v}_$rep.err; exit 1; }
    echo "$v $rep $(python -c "import json; d=json.load(open('gpurun_out/sw_${T}_${v}_$rep.json')); print(d['ms_per_step'], d['value'])")"
  done
done
