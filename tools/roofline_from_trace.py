"""Average duration of the roofline kernel (bridge.3's forward conv) in a rocprofv3 kernel trace
of `bench.py`, to set beside the bench line's HIP-event `launch_ms`.

    python tools/roofline_from_trace.py gpurun_out/prof_<tag>/bench_kernel_trace.csv [out.json]

Steps are delimited by the nchw_to_nhwc launch that starts every U-Net forward.  In forward
order the h3 256x128-tile launches of a step are enc2.conv1, enc2.conv2, enc3.conv1, enc3.conv2,
bridge.0, bridge.3, ... so bridge.3 is the 6th; its K-split tail fixup (the next launch, when
present) belongs to the same convolution and is added, as bench.py's events bracket both.
"""
import csv
import json
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "nchw_to_nhwc" in r["Kernel_Name"]]
durs = []
for a, b in zip(starts, starts[1:] + [len(rows)]):
    seen = 0
    for i in range(a, b):
        nm = rows[i]["Kernel_Name"]
        if "conv_fwd_h3_kernel<256, 128" in nm:
            seen += 1
            if seen == 6:
                d = int(rows[i]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"])
                if i + 1 < b and "conv_tail_fixup" in rows[i + 1]["Kernel_Name"]:
                    d = int(rows[i + 1]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"])
                durs.append(d / 1e6)
                break
# the first steps are warm-up; report all and the mean over the timed ones (all but the first 2)
rec = {"kernel": "conv_fwd_h3[bridge.3] (+ tail fixup)", "per_step_ms": [round(d, 4) for d in durs],
       "mean_ms_after_warmup": round(sum(durs[2:]) / max(1, len(durs[2:])), 4), "source": sys.argv[1]}
print(json.dumps(rec))
if len(sys.argv) > 2:
    json.dump(rec, open(sys.argv[2], "w"), indent=1)
