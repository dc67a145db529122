# per-layer conv table (time + PMC bytes) on this tree; DataParallel world 1 vs plain after the one-rank skip
#   gpurun -- bash tools/gpu/r04m.sh TAG
set -o pipefail
T=${1:-r04m}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_ddp.py tests/test_gpu_schedule.py -q --timeout 180 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1 || { tail -20 gpurun_out/pytest_$T.log; exit 1; }
tail -1 gpurun_out/pytest_$T.log
for rep in 1 2 3; do
  for v in plain ddp; do
    a=""; [ $v = ddp ] && a="--ddp"
    timeout -k 10 200 python bench.py $a --no-cpu-baseline --no-live-traffic --steps 20 --warmup 3 > gpurun_out/dp_${T}_${v}_$rep.json 2> gpurun_out/dp_${T}_${v}_$rep.err || { tail -5 gpurun_out/dp_${T}_${v}_$rep.err; exit 1; }
    echo "$v $rep $(python -c "import json,sys; print(json.load(open('gpurun_out/dp_${T}_${v}_$rep.json'))['ms_per_step'])")"
  done
done
bash tools/gpu/conv_table.sh $T || exit 1
cat gpurun_out/conv_layers_$T.md 2>/dev/null | head -60
