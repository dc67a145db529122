set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/finprof -o fwd -- python $R/tools/fwd_bench.py --mode train --iters 10 > $R/gpurun_out/finprof.log 2>&1 || { echo "prof failed"; tail -5 $R/gpurun_out/finprof.log; exit 1; }
cd $R
python - <<'PY'
import csv,glob,collections
f=glob.glob('gpurun_out/finprof/**/*kernel_trace.csv',recursive=True)[0]
rows=list(csv.DictReader(open(f)))
d=collections.defaultdict(list)
for r in rows:
    n=r['Kernel_Name']
    if 'finalize' in n or 'stats_split' in n:
        d[(n[:40], r['Grid_Size_X'], r['Grid_Size_Y'])].append((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1000)
for k,v in sorted(d.items()): print(k, len(v), round(sum(v)/len(v),2))
PY
