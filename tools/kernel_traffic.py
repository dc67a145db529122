"""HBM bytes per dispatch of every kernel name in rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs):
FETCH_SIZE x2 (gfx950: half the bytes of wide streaming reads, MI355X_MICROARCH.md HBM section) + WRITE_SIZE,
KiB -> B.  Names are normalised to what srpde_last_kernel reports ("conv_fwd_h5_kernel<2, 8>").
    python tools/kernel_traffic.py DIR  -> one JSON line {name: {"dispatches": n, "bytes_per_dispatch": b, ...}}"""
import collections
import csv
import glob
import json
import re
import sys


def norm(k):
    k = re.sub(r"^void ", "", k)
    k = k.replace("srpde::", "")
    i, depth = 0, 0
    for i, ch in enumerate(k):   # drop the parameter list: the first '(' outside template brackets
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return k[:i].strip()
    return k.strip()


def main():
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[norm(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in acc.items():
        fe, wr = cs.get("FETCH_SIZE", []), cs.get("WRITE_SIZE", [])
        if not fe or not wr:
            continue
        rb = 2 * 1024 * sum(fe) / len(fe)
        wb = 1024 * sum(wr) / len(wr)
        out[k] = {"dispatches": len(fe), "bytes_per_dispatch": round(rb + wb), "read_bytes": round(rb),
                  "write_bytes": round(wb)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
