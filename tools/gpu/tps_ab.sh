set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for rep in 1 2; do for t in 2 1; do
SRPDE_H3_TPS=$t timeout -k 10 200 python tools/conv_bench.py --iters 10 --only fwd,dgrad --json-out gpurun_out/tps_${t}_$rep.json > gpurun_out/tps_${t}_$rep.log 2>&1 || exit 1
done; done
python - <<'P'
import json,glob
for t in (2,1):
    rows={}
    for f in glob.glob(f"gpurun_out/tps_{t}_*.json"):
        for r in json.load(open(f))["rows"]:
            k=(r["layer"],r["pass"]); rows[k]=min(rows.get(k,1e9), r["ms"])
    print(t, round(sum(rows.values()),3), {k[0]+":"+k[1]: v for k,v in rows.items() if k[0] in ("enc1.conv2","bridge.3","dec1.conv1","dec2.conv1")})
P
