"""Micro-benchmark of the HIP conv kernels per U-Net layer at batch 1024 (fwd, dgrad, wgrad).

    python tools/conv_bench.py [--batch 1024] [--iters 10] [--only fwd|dgrad|wgrad]
Prints TFLOP/s per layer and the FLOP-weighted total for each pass.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from superresolution_for_pdes_amd import hipops as H  # noqa: E402

# (name, c0, c1, cout, hw, dil)
LAYERS = [("enc1.conv2", 64, 0, 64, 40, 1), ("enc2.conv1", 64, 0, 128, 20, 1), ("enc2.conv2", 128, 0, 128, 20, 1),
          ("enc3.conv1", 128, 0, 256, 10, 1), ("enc3.conv2", 256, 0, 256, 10, 1), ("bridge.0", 256, 0, 512, 10, 2),
          ("bridge.3", 512, 0, 512, 10, 2), ("dec3.conv1", 512, 256, 256, 10, 1), ("dec3.conv2", 256, 0, 256, 10, 1),
          ("dec2.conv1", 256, 128, 128, 20, 1), ("dec2.conv2", 128, 0, 128, 20, 1), ("dec1.conv1", 128, 64, 64, 40, 1),
          ("dec1.conv2", 64, 0, 64, 40, 1), ("out_conv1", 64, 0, 32, 40, 1), ("out_conv2", 32, 0, 16, 40, 1)]


def timeit(fn, iters, seq=None, tag=None):
    if seq is not None:
        seq.extend([tag] * (iters + 2))
    for _ in range(2):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="fwd,dgrad,wgrad")
    ap.add_argument("--layers", default="")
    ap.add_argument("--math", default=None, choices=("h3", "f32"), help="default: the package default (h3)")
    ap.add_argument("--json-out", default=None, help="per (layer, pass): ms, TF, algorithmic bytes")
    ap.add_argument("--sequence-out", default=None,
                    help="launch order of every conv call [(layer, pass)] (maps rocprofv3 dispatches to layers)")
    args = ap.parse_args()
    seq, rows = [], []
    if args.math:
        H.set_conv_math(args.math)
    dev = "cuda"
    n = args.batch
    tot = {}
    for name, c0, c1, cout, hw, dil in LAYERS:
        if args.layers and name not in args.layers.split(","):
            continue
        cin = c0 + c1
        P = n * hw * hw
        flops = 2.0 * cout * cin * 9 * P
        x = torch.randn(P, cin, device=dev)
        x0, x1 = (x[:, :c0], x[:, c0:]) if c1 else (x, None)
        w = torch.randn(cout, cin, 3, 3, device=dev) * 0.05
        b = torch.randn(cout, device=dev)
        wf, wd = H.pack_conv_weights(w, cin, True, True)
        y = torch.empty(P, cout, device=dev)
        stats, _, _ = H.conv_stats_buffer(n, hw, hw, cout, dev, c0, c1, dil)
        dy = torch.randn(P, cout, device=dev)
        for t in (x0, x1, dy):   # h3: max|x| words computed once, as the producers would
            if t is not None:
                t._srpde_amax = H.amax_of(t)
        dx = torch.empty(P, cin, device=dev)
        dw = torch.empty_like(w)
        line = f"{name:11s}"
        # h3 as training runs it: the forward stores its input split, the dgrad reads dy as split planes
        # (bn_bwd_apply_split's output, 32-channel padded for out_conv2) and the wgrad reads both
        cp = H.cpad32(cout)
        h3p = H.conv_math() == "h3" and H.h3_capable(c0, c1, cout, hw, dil) and H.h3_capable(cp, 0, cin, hw, dil)
        # the 40 x 40 layers as training runs them: no stored input split, the weight gradient splits the
        # fp32 rows itself (srpde_conv_wgrad_h3x; unet_exec._WGRAD_X)
        wx = h3p and H.wgrad_x_capable(c0, c1, cout, hw, dil)
        xp = H.split_planes_buffer(P, cin, dev) if h3p else None
        dyp = H.split_planes_buffer(P, cp, dev) if h3p else None
        xfwd = None if wx else xp
        if h3p:
            dyin = dy if cp == cout else torch.cat([dy, torch.zeros(P, cp - cout, device=dev)], 1)
            dyin._srpde_amax = dy._srpde_amax
            H.conv_fwd(x0, x1, wf, b, y, n, hw, hw, cout, 3, dil, 1, False, stats, xp)
            H.conv_fwd(dyin, None, wd, None, dx, n, hw, hw, cin, 3, dil, -1, False, None, dyp)
            seq.extend([(name, "setup"), (name, "setup")])
            if wx:
                xp = H.XSource(x0, x1, None, None)
        for kind in args.only.split(","):
            tag = (name, kind)
            if kind == "fwd":
                ms = timeit(lambda: H.conv_fwd(x0, x1, wf, b, y, n, hw, hw, cout, 3, dil, 1, False, stats, xfwd),
                            args.iters, seq, tag)
            elif kind == "dgrad" and h3p:
                ms = timeit(lambda: H.conv_fwd_presplit(dyp, wd, None, dx, n, hw, hw, cin, 3, dil, -1), args.iters,
                            seq, tag)
            elif kind == "dgrad":
                ms = timeit(lambda: H.conv_fwd(dy, None, wd, None, dx, n, hw, hw, cin, 3, dil, -1), args.iters, seq,
                            tag)
            elif h3p:
                ms = timeit(lambda: H.conv_wgrad_h3p(dyp, xp, dw, n, hw, hw, 3, dil), args.iters, seq, tag)
            else:
                ms = timeit(lambda: H.conv_wgrad(dy, x0, x1, dw, n, hw, hw, 3, dil), args.iters, seq, tag)
            tf = flops / ms / 1e9
            # algorithmic HBM bytes of one call (fp32 4 B/elem; stored h3 splits 2x2 B/elem):
            # fwd x + w + y (+ the input split it stores, not at the 40 x 40 layers); dgrad dy + w + dx
            # (+ dy's split); wgrad: both operands (stored splits or fp32: 4 B/elem either way) + dw
            wb = 4 * cout * cin * 9
            if kind == "fwd":
                ab = 4 * P * cin + wb + 4 * P * cout + (4 * P * cin if h3p and not wx else 0)
            elif kind == "dgrad":   # h3: dy arrives as its stored split (4 B/elem), nothing else stored
                ab = 4 * P * cout + wb + 4 * P * cin
            else:
                ab = 4 * P * (cin + cout) + wb
            rows.append({"layer": name, "pass": kind, "ms": round(ms, 4), "tflops": round(tf, 1), "flop": flops,
                         "algorithmic_bytes": ab, "h3p": h3p, "wgrad_x": wx})
            t = tot.setdefault(kind, [0.0, 0.0])
            t[0] += flops
            t[1] += ms
            line += f"  {kind} {ms:7.3f} ms {tf:6.1f} TF"
        print(line, flush=True)
    for k, (f, ms) in tot.items():
        print(f"TOTAL {k}: {ms:.2f} ms  {f / ms / 1e9:.1f} TF/s")
    import json
    if args.json_out:
        json.dump({"batch": n, "math": H.conv_math(), "rows": rows,
                   "totals": {k: {"ms": round(ms, 3), "tflops": round(f / ms / 1e9, 1)} for k, (f, ms) in tot.items()}},
                  open(args.json_out, "w"), indent=1)
    if args.sequence_out:
        json.dump(seq, open(args.sequence_out, "w"))


if __name__ == "__main__":
    main()
