"""Per-stream busy time of one training step in a rocprofv3 kernel trace of bench.py (the wgrad
side stream overlaps the compute stream): span, union busy, busy per stream, and the compute
stream's largest kernels.   python tools/stream_split.py gpurun_out/prof_<tag>/bench_kernel_trace.csv [step]"""
import collections
import csv
import sys


def union(iv):
    tot, cs, ce = 0, None, None
    for s, e in sorted(iv):
        if cs is None:
            cs, ce = s, e
        elif s <= ce:
            ce = max(ce, e)
        else:
            tot += ce - cs
            cs, ce = s, e
    return tot + (ce - cs if cs is not None else 0)


rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 4
starts = [i for i, r in enumerate(rows) if "nchw_to_nhwc" in r["Kernel_Name"]]
step = rows[starts[k]:starts[k + 1]]
iv = lambda rs: [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rs]  # noqa: E731
t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
print(f"step {k}: span {(t1 - t0) / 1e6:.3f} ms, union busy {union(iv(step)) / 1e6:.3f} ms")
streams = collections.Counter(r["Stream_Id"] for r in step)
for sid, cnt in streams.most_common():
    print(f"  stream {sid}: {cnt} launches, busy {union(iv([r for r in step if r['Stream_Id'] == sid])) / 1e6:.3f} ms")
main = streams.most_common(1)[0][0]
tot = collections.Counter()
for r in step:
    if r["Stream_Id"] == main:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("srpde::", "")[:60]
        tot[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
for name, ms in tot.most_common(16):
    print(f"  {ms:7.3f}  {name}")
