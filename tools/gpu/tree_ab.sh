# Same-box bench of earlier trees (git worktrees with their own built library, e.g. ab_r05/, ab_r06b/) against this
# one, interleaved:   gpurun -- bash tools/gpu/tree_ab.sh TAG REPS DIR...
set -o pipefail
T=$1; N=$2; shift 2
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
for rep in $(seq 1 $N); do
  for v in "$@" .; do
    tag=$(basename $(cd $v && pwd))
    (cd $v && timeout -k 10 200 python bench.py --no-cpu-baseline --no-live-traffic --steps 20 --warmup 3) > gpurun_out/tab_${T}_${tag}_$rep.json 2> gpurun_out/tab_${T}_${tag}_$rep.err || { echo "bench $v failed"; tail gpurun_out/tab_${T}_${tag}_$rep.err; exit 1; }
    echo "$v $rep $(python -c "import json; d=json.load(open('gpurun_out/tab_${T}_${tag}_$rep.json')); f=d['roofline']['forward']; print(d['ms_per_step'], d['value'], f['eval']['ms'], f['train']['ms'])")"
  done
done
