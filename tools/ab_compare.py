"""Same-box A/B of tools/conv_bench.py runs: PREFIX_{base,new}_{1,2}.json -> per (layer, pass) best-of-2 ms."""
import glob
import json
import sys

pre = sys.argv[1]
best = {}
for v in ("base", "new"):
    for f in sorted(glob.glob(f"{pre}_{v}_*.json")):
        for r in json.load(open(f))["rows"]:
            k = (r["layer"], r["pass"])
            best.setdefault(v, {})
            best[v][k] = min(best[v].get(k, 1e9), r["ms"])
tb = tn = 0.0
print(f"{'layer':12s} {'pass':6s} {'base ms':>8s} {'new ms':>8s} {'delta':>7s}")
for k in best["base"]:
    b, n = best["base"][k], best["new"].get(k)
    tb += b
    tn += n
    print(f"{k[0]:12s} {k[1]:6s} {b:8.3f} {n:8.3f} {100 * (n / b - 1):+6.1f}%")
print(f"{'TOTAL':19s} {tb:8.3f} {tn:8.3f} {100 * (tn / tb - 1):+6.1f}%")
