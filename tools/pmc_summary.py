"""Average PMC counters per dispatch for kernels matching a substring (rocprofv3 csv dirs)."""
import csv, glob, sys, collections
d, pat = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "conv"
acc = collections.defaultdict(list)
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(acc):
    v = acc[k]
    print(f"{k:28s} n={len(v):3d} mean={sum(v)/len(v):.4g}")
