# Kernel traces of the bench step for two settings of one env knob, same box:
#   gpurun -- bash tools/gpu/trace_ab.sh TAG VAR VALUE_A VALUE_B
set -o pipefail
T=$1; V=$2; A=$3; B=$4
R=$GRAFT_REPO_ROOT
cd /tmp
export TMPDIR=/tmp
for val in $A $B; do
  export $V=$val
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/tr_${T}_$val -o b -- python $R/bench.py --steps 7 --warmup 3 --no-cpu-baseline > $R/gpurun_out/tr_${T}_$val.log 2>&1 || { echo "trace $val failed"; tail -5 $R/gpurun_out/tr_${T}_$val.log; exit 1; }
done
cd $R
for val in $A $B; do
  echo "== $V=$val"
  f=$(ls gpurun_out/tr_${T}_$val/*kernel_trace.csv | head -1)
  python tools/stream_split.py $f 5 | head -24
done
