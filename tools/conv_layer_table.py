"""Per-conv-layer table: achieved TFLOP/s and PMC HBM traffic for fwd / dgrad / wgrad at batch 1024.

    python tools/conv_layer_table.py TIMING.json SEQUENCE.json PMC_FETCH_DIR PMC_WRITE_DIR OUT_PREFIX

TIMING.json / SEQUENCE.json: tools/conv_bench.py --json-out / --sequence-out of the timing run and
of the PMC runs (same arguments, so the same launch order).  rocprofv3 dispatches are grouped into
calls -- a conv main kernel (srpde::conv_*_kernel) plus the helpers that follow it (tail fixup,
split-K reduce) -- in Dispatch_Id order and zipped with the sequence.  HBM bytes per call =
2 x FETCH_SIZE + WRITE_SIZE (KiB; the gfx950 FETCH_SIZE halving of wide streaming reads,
MI355X_MICROARCH.md HBM section), averaged over the timed calls of that (layer, pass).
Writes OUT_PREFIX.json and OUT_PREFIX.md.
"""
import collections
import csv
import glob
import json
import re
import sys

MAIN = re.compile(r"srpde::conv_\w+_kernel")
PEAK_TF = 838.9          # h3 roof: 2516.8 TF fp16 MFMA / 3 products
PEAK_GBS = 8000.0


def dispatch_calls(d, counter):
    rows = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    rows.sort()
    calls = []
    for _, name, v in rows:
        if MAIN.search(name) and "tail_fixup" not in name:
            calls.append(v)
        elif calls and ("fixup" in name or "reduce" in name):
            calls[-1] += v
    return calls


def main():
    timing, seq_f, dfetch, dwrite, out = sys.argv[1:6]
    tim = json.load(open(timing))
    seq = [tuple(s) for s in json.load(open(seq_f))]
    fetch = dispatch_calls(dfetch, "FETCH_SIZE")
    write = dispatch_calls(dwrite, "WRITE_SIZE")
    if len(fetch) != len(seq) or len(write) != len(seq):
        raise SystemExit(f"dispatch groups {len(fetch)}/{len(write)} != sequence {len(seq)}")
    acc = collections.defaultdict(list)
    for i, tag in enumerate(seq):
        acc[tag].append(2 * 1024 * fetch[i] + 1024 * write[i])
    table = []
    for r in tim["rows"]:
        b = acc.get((r["layer"], r["pass"]), [])
        b = b[2:] if len(b) > 2 else b          # skip the two warm-up calls
        hbm = sum(b) / len(b) if b else None
        t = r["ms"] * 1e-3
        table.append(dict(r, hbm_bytes=round(hbm) if hbm else None,
                          hbm_gbs=round(hbm / t / 1e9, 1) if hbm else None,
                          traffic_over_algorithmic=round(hbm / r["algorithmic_bytes"], 2) if hbm else None,
                          mfma_frac=round(r["tflops"] / PEAK_TF, 3)))
    json.dump({"batch": tim["batch"], "math": tim["math"], "peak_tflops": PEAK_TF, "rows": table,
               "totals": tim["totals"]}, open(out + ".json", "w"), indent=1)
    with open(out + ".md", "w") as f:
        f.write(f"Per-layer conv kernels, batch {tim['batch']}, {tim['math']} (roof {PEAK_TF} TF); HBM = 2xFETCH_SIZE + "
                "WRITE_SIZE per call (rocprofv3 PMC), algorithmic = operands + outputs + stored splits.\n\n")
        f.write("| layer | pass | ms | TFLOP/s | frac of roof | HBM MB | HBM GB/s | HBM / algorithmic |\n")
        f.write("|---|---|---|---|---|---|---|---|\n")
        for r in table:
            mb = f"{r['hbm_bytes'] / 1e6:.1f}" if r["hbm_bytes"] else "-"
            f.write(f"| {r['layer']} | {r['pass']} | {r['ms']:.3f} | {r['tflops']:.1f} | {r['mfma_frac']:.3f} | {mb} | "
                    f"{r['hbm_gbs'] or '-'} | {r['traffic_over_algorithmic'] or '-'} |\n")
        for k, v in tim["totals"].items():
            f.write(f"\nTOTAL {k}: {v['ms']} ms, {v['tflops']} TF/s")
        f.write("\n")
    print(open(out + ".md").read())


if __name__ == "__main__":
    main()
