"""Average SQ counters per dispatch of the conv main kernels (or the kernels matching PATTERN),
grouped by (kernel, grid size) (distinguishes layers of one instantiation).
    python tools/pmc_by_grid.py DIR [PATTERN]"""
import collections
import csv
import glob
import re
import sys

pat = sys.argv[2] if len(sys.argv) > 2 else r"srpde::conv_\w+_kernel"
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if not re.search(pat, k) or "fixup" in k:
            continue
        key = (re.sub(r"\(.*", "", k).replace("void srpde::", ""), r.get("Grid_Size", "?"))
        acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for key, cs in acc.items():
    print(key)
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    for c in sorted(m):
        print(f"   {c:28s} {m[c]:.4g}")
    if "SQ_INSTS_MFMA" in m and m["SQ_INSTS_MFMA"]:
        print(f"   VALU/MFMA {m.get('SQ_INSTS_VALU', 0) / m['SQ_INSTS_MFMA']:.2f}  SALU/MFMA "
              f"{m.get('SQ_INSTS_SALU', 0) / m['SQ_INSTS_MFMA']:.2f}  LDS/MFMA {m.get('SQ_INSTS_LDS', 0) / m['SQ_INSTS_MFMA']:.2f}")
    if "SQ_WAVE_CYCLES" in m:
        w = m["SQ_WAVE_CYCLES"]
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                  "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_VMEM", "SQ_WAIT_INST_LDS"):
            if c in m:
                print(f"   {c} / WAVE_CYCLES = {m[c] / w:.3f}")
