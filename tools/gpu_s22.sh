# Weight gradients on the side stream (default) vs in line on the compute stream.
set -o pipefail
T=${1:-s22}
cd $GRAFT_REPO_ROOT
for v in side inline side2 inline2; do
  case $v in side*) W=1;; *) W=0;; esac
  SRPDE_WGRAD_STREAM=$W timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_${T}_$v.json 2> gpurun_out/bench_${T}_$v.err || { echo "$v failed"; exit 1; }
  echo "$v: $(python -c "import json; d=json.load(open('gpurun_out/bench_${T}_$v.json')); print(d['ms_per_step'], d['value'], d['roofline']['launch_ms'])")"
done
