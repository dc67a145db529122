"""Per-kernel total time of two rocprofv3 --stats runs (e.g. baseline vs new build), largest differences first.
    python tools/kstats_diff.py DIR_A DIR_B"""
import csv
import glob
import re
import sys


def load(d):
    f = glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True)[0]
    out = {}
    for r in csv.DictReader(open(f)):
        name = re.sub(r"\(.*", "", r["Name"]).replace("void ", "").replace("srpde::", "")
        out[name] = out.get(name, 0.0) + float(r["TotalDurationNs"]) / 1e6
    return out


a, b = load(sys.argv[1]), load(sys.argv[2])
rows = sorted(set(a) | set(b), key=lambda k: -abs(b.get(k, 0) - a.get(k, 0)))
print(f"{'kernel':70s} {'A ms':>9s} {'B ms':>9s} {'B-A':>8s}")
for k in rows[:25]:
    print(f"{k[:70]:70s} {a.get(k, 0):9.3f} {b.get(k, 0):9.3f} {b.get(k, 0) - a.get(k, 0):8.3f}")
print(f"{'TOTAL':70s} {sum(a.values()):9.3f} {sum(b.values()):9.3f} {sum(b.values()) - sum(a.values()):8.3f}")
