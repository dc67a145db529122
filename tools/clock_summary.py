"""GRBM_GUI_ACTIVE / kernel duration per dispatch (effective clock) from a rocprofv3 pmc dir."""
import csv, glob, sys
d, pat = sys.argv[1], sys.argv[2]
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    rows = [r for r in csv.DictReader(open(f)) if pat in r["Kernel_Name"]]
    for r in rows:
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9 if "End_Timestamp" in r else None
        print(f"{r['Kernel_Name'][:50]:50s} {r['Counter_Name']:16s} {float(r['Counter_Value']):.4g}"
              + (f"  dur {dur*1e3:.3f} ms  -> {float(r['Counter_Value'])/dur/1e9:.3f} GHz" if dur and 'GUI' in r['Counter_Name'] else ""))
