"""Attribute the raw frame addresses of a crash report ("@ 0x... ") to the objects of a saved
/proc/<pid>/maps:  python tools/attribute_frames.py CRASH_LOG MAPS"""
import re
import sys

log, maps = sys.argv[1], sys.argv[2]
regions = []
try:
    for line in open(maps):
        f = line.split()
        lo, hi = (int(v, 16) for v in f[0].split("-"))
        regions.append((lo, hi, int(f[2], 16), f[5] if len(f) > 5 else "[anon]"))
except FileNotFoundError:
    print("no maps file (the process did not reach Python exit)")
    sys.exit(0)
frames = re.findall(r"(?:PC:|@)\s+(0x[0-9a-f]+)\s*(\S*)", open(log, errors="replace").read())
if not frames:
    print("no crash frames in the log")
for a, sym in frames:
    v = int(a, 16)
    hit = next(((lo, off, name) for lo, hi, off, name in regions if lo <= v < hi), None)
    if hit:
        lo, off, name = hit
        print(f"{a}  {name} + {v - lo + off:#x}  {sym}")
    else:
        print(f"{a}  (unmapped)  {sym}")
