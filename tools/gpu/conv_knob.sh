# Per-layer conv timing under several settings of one env knob, same box, interleaved twice:
#   gpurun -- bash tools/gpu/conv_knob.sh TAG VAR "v1 v2 ..." [LAYERS] [PASSES]
set -o pipefail
T=$1; V=$2; VALS=$3; L=${4:-}; K=${5:-fwd,dgrad,wgrad}
R=$GRAFT_REPO_ROOT
cd $R
LA=""
[ -n "$L" ] && LA="--layers $L"
for rep in 1 2; do
  for val in $VALS; do
    timeout -k 10 300 env $V=$val python tools/conv_bench.py --iters 10 --only $K $LA --json-out gpurun_out/ck_${T}_${val}_$rep.json > gpurun_out/ck_${T}_${val}_$rep.log 2>&1 || { echo "bench $val failed"; tail gpurun_out/ck_${T}_${val}_$rep.log; exit 1; }
  done
done
for val in $VALS; do echo "== $V=$val"; grep -v "^$" gpurun_out/ck_${T}_${val}_2.log | tail -20; done
