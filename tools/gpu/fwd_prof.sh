# Forward-only kernel summaries (north_star's roofline target): rocprofv3 --kernel-trace --stats of
# tools/fwd_bench.py in eval and train mode, 10 forwards + 3 warm-ups each.
#   gpurun -- bash tools/gpu/fwd_prof.sh TAG      -> gpurun_out/fwdprof_TAG_{eval,train}/...
set -o pipefail
T=${1:-t}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
for M in eval train; do
  timeout -k 10 120 python tools/fwd_bench.py --mode $M --iters 20 > gpurun_out/fwd_${T}_$M.json 2> gpurun_out/fwd_${T}_$M.err || { echo "fwd $M failed"; tail -5 gpurun_out/fwd_${T}_$M.err; exit 1; }
  cat gpurun_out/fwd_${T}_$M.json
done
cd /tmp
for M in eval train; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/fwdprof_${T}_$M -o fwd -- python $R/tools/fwd_bench.py --mode $M --iters 10 > $R/gpurun_out/fwdprof_${T}_$M.log 2>&1 || { echo "prof $M failed"; tail -5 $R/gpurun_out/fwdprof_${T}_$M.log; exit 1; }
done
cd $R
for M in eval train; do
  f=$(find gpurun_out/fwdprof_${T}_$M -name "*kernel_stats.csv" | head -1)
  echo "== $M"; python tools/kstats.py $f 13 30
done
