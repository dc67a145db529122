# config #5 cascade line on the cascade20 bounded weights (with the reference-output check and the CPU
# baseline); DataParallel at world 1 against the plain step (interleaved, same box) and the stream
# split of each from a kernel trace
#   gpurun -- bash tools/gpu/r04l.sh TAG
set -o pipefail
T=${1:-r04l}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
python -c "import sys, torch; sys.path.insert(0, 'tests/golden'); from state import fixture_state_torch; torch.save(fixture_state_torch(), 'gpurun_out/cascade20_state.pt')" || exit 1
timeout -k 10 400 python bench.py --workload cascade --checkpoint gpurun_out/cascade20_state.pt \
  --cascade-fixture tests/golden/cascade640_fixture.npz --steps 10 --warmup 2 > gpurun_out/cascade_$T.json 2> gpurun_out/cascade_$T.err || { tail -5 gpurun_out/cascade_$T.err; exit 1; }
cat gpurun_out/cascade_$T.json
for rep in 1 2 3; do
  for v in plain ddp; do
    a=""; [ $v = ddp ] && a="--ddp"
    timeout -k 10 200 python bench.py $a --no-cpu-baseline --no-live-traffic --steps 20 --warmup 3 > gpurun_out/dp_${T}_${v}_$rep.json 2> gpurun_out/dp_${T}_${v}_$rep.err || { tail -5 gpurun_out/dp_${T}_${v}_$rep.err; exit 1; }
    echo "$v $rep $(python -c "import json,sys; print(json.load(open('gpurun_out/dp_${T}_${v}_$rep.json'))['ms_per_step'])")"
  done
done
cd /tmp
for v in plain ddp; do
  a=""; [ $v = ddp ] && a="--ddp"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/dptrace_${T}_$v -o bench -- python $R/bench.py $a --no-cpu-baseline --no-live-traffic --steps 8 --warmup 3 > $R/gpurun_out/dptrace_${T}_$v.log 2>&1 || { tail -5 $R/gpurun_out/dptrace_${T}_$v.log; exit 1; }
done
cd $R
for v in plain ddp; do
  f=$(find gpurun_out/dptrace_${T}_$v -name "*kernel_trace.csv" | head -1)
  echo "== $v"; python tools/stream_split.py $f 6 | head -12
done
