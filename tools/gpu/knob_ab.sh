# Train-step timing of env-knob variants on ONE box, interleaved:
#   gpurun -- bash tools/gpu/knob_ab.sh TAG REPS "VAR1=a VAR2=b" "VAR1=c" ...   (pytest -k selector in PYK, optional)
set -o pipefail
T=$1; N=$2; shift 2
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
if [ -n "$PYK" ]; then
  timeout -k 10 500 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "$PYK" > gpurun_out/knob_pytest_$T.log 2>&1 || { echo "tests failed"; grep -v amdgpu gpurun_out/knob_pytest_$T.log | tail -30; exit 1; }
  tail -1 gpurun_out/knob_pytest_$T.log
fi
for rep in $(seq 1 $N); do
  i=0
  for cfg in "$@"; do
    i=$((i+1))
    env $cfg timeout -k 10 200 python bench.py --no-cpu-baseline --no-live-traffic --steps 20 > gpurun_out/knob_${T}_${i}_$rep.json 2> gpurun_out/knob_${T}_${i}_$rep.err || { echo "bench [$cfg] failed"; tail gpurun_out/knob_${T}_${i}_$rep.err; exit 1; }
    echo "[$cfg] $rep $(python -c "import json; d=json.load(open('gpurun_out/knob_${T}_${i}_$rep.json')); print(d['ms_per_step'], d['value'])")"
  done
done
