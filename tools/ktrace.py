"""Per-dispatch view of the last step in a rocprofv3 kernel_trace.csv (conv kernels annotated
with grid size so layers can be told apart)."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# a step starts at the first nchw_to_nhwc launch
starts = [i for i, r in enumerate(rows) if "nchw_to_nhwc" in r["Kernel_Name"]]
a = starts[-2]; b = starts[-1]
t0 = int(rows[a]["Start_Timestamp"])
tot = 0
for r in rows[a:b]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    nm = r["Kernel_Name"].split("(")[0].replace("void srpde::", "").replace("srpde::", "")
    if d > float(sys.argv[2] if len(sys.argv) > 2 else 50):
        print(f"{(int(r['Start_Timestamp'])-t0)/1e3:9.1f}us {d:9.1f}us grid={r['Grid_Size_X']:>8s} {nm}")
print(f"busy {tot/1e3:.2f} ms, wall {(int(rows[b]['Start_Timestamp'])-t0)/1e6:.2f} ms")
