"""Same-process A/B of the h5 kernel (conv_h5.hip) against h4 / h3r on the U-Net's 40x40 convolutions and on
the whole B=1024 forward:  python tools/h5_ab.py [--reps 3] [--batch 1024] [--layers] [--forward]

Per layer (batch 1024): the eval-mode forward (BN + ReLU epilogue, the gated input of dec1.conv1) and the
training forward (statistics + stored split, fused input BN / gated input), ms and TF/s (h3 roof 838.9 TF),
h5 off / on interleaved --reps times.  --forward: bench.py's eval / train forward timing with h5 off / on."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

LAYERS = [("enc1.conv2", 64, 0, 64), ("dec1.conv1", 128, 64, 64), ("dec1.conv2", 64, 0, 64), ("out_conv1", 64, 0, 32)]


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def layers(H, n, reps):
    dev = "cuda"
    hw = 40
    P = n * hw * hw
    res = {}
    for name, c0, c1, cout in LAYERS:
        cin = c0 + c1
        flops = 2.0 * cout * cin * 9 * P
        g = torch.Generator(device=dev).manual_seed(1)
        x = torch.randn(P, cin, device=dev, generator=g)
        x0, x1 = (x[:, :c0], x[:, c0:]) if c1 else (x, None)
        w = torch.randn(cout, cin, 3, 3, device=dev, generator=g) * 0.05
        b = torch.randn(cout, device=dev, generator=g)
        wf, _ = H.pack_conv_weights(w, cin, True, False)
        for t in (x0, x1):
            if t is not None:
                t._srpde_amax = H.amax_of(t)
        ep = (torch.zeros(cout, device=dev), torch.ones(cout, device=dev), torch.ones(cout, device=dev),
              torch.zeros(cout, device=dev), torch.zeros(1, dtype=torch.int32, device=dev))
        gate = None
        aff = None
        if c1:
            gate = (torch.sigmoid(torch.randn(n, c1, device=dev, generator=g)),
                    torch.sigmoid(torch.randn(P, device=dev, generator=g)))
        else:
            aff = (torch.rand(c0, device=dev, generator=g) + 0.5, torch.randn(c0, device=dev, generator=g) * 0.2)
        y = torch.empty(P, cout, device=dev)
        xp = H.split_planes_buffer(P, cin, dev)
        for rep in range(reps):
            for on in (False, True):
                H.set_h5(on)
                stats, _, _ = H.conv_stats_buffer(n, hw, hw, cout, dev, c0, c1, 1)
                ev = timeit(lambda: H.conv_fwd(x0, x1, wf, b, y, n, hw, hw, cout, 3, 1, 1, False, None, ep_bn=ep,
                                               x1_gate=gate))
                tr = timeit(lambda: H.conv_fwd(x0, x1, wf, b, y, n, hw, hw, cout, 3, 1, 1, False, stats, xp,
                                               in_affine=aff, x1_gate=gate))
                key = f"{name} h5={int(on)}"
                r = res.setdefault(key, {"eval_ms": [], "train_ms": [], "flop": flops})
                r["eval_ms"].append(round(ev, 4))
                r["train_ms"].append(round(tr, 4))
        H.set_h5(True)
    for k, r in res.items():
        ev, tr = min(r["eval_ms"]), min(r["train_ms"])
        print(f"{k:18s} eval {ev:7.3f} ms {r['flop'] / ev / 1e9:6.1f} TF ({r['flop'] / ev / 1e9 / 838.9:.3f})   "
              f"train {tr:7.3f} ms {r['flop'] / tr / 1e9:6.1f} TF ({r['flop'] / tr / 1e9 / 838.9:.3f})", flush=True)
    return res


def forward(H, n, reps):
    import bench
    from superresolution_for_pdes_amd.models import UNet, init_weights
    dev = torch.device("cuda", 0)
    torch.manual_seed(42)
    model = UNet()
    model.apply(init_weights)
    model = model.to(dev)
    g = torch.Generator(device=dev).manual_seed(1234)
    x = torch.randn(n, 3, 40, 40, device=dev, generator=g)
    x[:, 1] = 1.0
    res = {}
    for rep in range(reps):
        for on in (False, True):
            H.set_h5(on)
            for mode in ("eval", "train"):
                ms = bench.time_forward(model, x, mode == "train", reps=10, warm=3)
                res.setdefault(f"{mode} h5={int(on)}", []).append(round(ms, 4))
    H.set_h5(True)
    for k, v in res.items():
        print(f"forward {k:12s} {min(v):7.3f} ms  (all: {v})", flush=True)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--layers", action="store_true")
    ap.add_argument("--forward", action="store_true")
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()
    from superresolution_for_pdes_amd import hipops as H
    out = {}
    if a.layers or not a.forward:
        out["layers"] = layers(H, a.batch, a.reps)
    if a.forward:
        out["forward"] = forward(H, a.batch, a.reps)
    if a.json_out:
        json.dump(out, open(a.json_out, "w"), indent=1)


if __name__ == "__main__":
    main()
