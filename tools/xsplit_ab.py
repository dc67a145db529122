"""What the stored input split costs the 40x40 training forwards: the same launch with and without
the split planes (statistics either way), plus the h3h weight gradient that reads them.
    python tools/xsplit_ab.py [--reps 3] [--batch 1024]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

LAYERS = [("enc1.conv2", 64, 0, 64), ("dec1.conv1", 128, 64, 64), ("dec1.conv2", 64, 0, 64), ("out_conv1", 64, 0, 32),
          ("out_conv2", 32, 0, 16)]
# the deeper layers (h4 forwards; their weight gradients are h3p): (name, c0, c1, cout, hw, dil)
DEEP = [("enc2.conv1", 64, 0, 128, 20, 1), ("enc2.conv2", 128, 0, 128, 20, 1), ("enc3.conv1", 128, 0, 256, 10, 1),
        ("enc3.conv2", 256, 0, 256, 10, 1), ("bridge.0", 256, 0, 512, 10, 2), ("bridge.3", 512, 0, 512, 10, 2),
        ("dec3.conv1", 512, 256, 256, 10, 1), ("dec3.conv2", 256, 0, 256, 10, 1), ("dec2.conv1", 256, 128, 128, 20, 1),
        ("dec2.conv2", 128, 0, 128, 20, 1)]


def deep(H, n, reps):
    """plain training forward with / without the stored split at the deeper layers"""
    dev = "cuda"
    tot = [0.0, 0.0]
    for name, c0, c1, cout, hw, dil in DEEP:
        cin, P = c0 + c1, n * hw * hw
        g = torch.Generator(device=dev).manual_seed(2)
        x = torch.relu(torch.randn(P, cin, device=dev, generator=g))
        x0, x1 = (x[:, :c0], x[:, c0:]) if c1 else (x, None)
        w = torch.randn(cout, cin, 3, 3, device=dev, generator=g) * 0.05
        b = torch.randn(cout, device=dev, generator=g)
        wf, _ = H.pack_conv_weights(w, cin, True, False)
        for t in (x0, x1):
            if t is not None:
                t._srpde_amax = H.amax_of(t)
        y = torch.empty(P, cout, device=dev)
        xp = H.split_planes_buffer(P, cin, dev)
        stats, _, _ = H.conv_stats_buffer(n, hw, hw, cout, dev, c0, c1, dil)
        a, bb = [], []
        for _ in range(reps):
            a.append(timeit(lambda: H.conv_fwd(x0, x1, wf, b, y, n, hw, hw, cout, 3, dil, 1, False, stats, xp)))
            bb.append(timeit(lambda: H.conv_fwd(x0, x1, wf, b, y, n, hw, hw, cout, 3, dil, 1, False, stats, None)))
        tot[0] += min(a)
        tot[1] += min(bb)
        print(f"{name:11s}  split {min(a):7.3f} ms  nosplit {min(bb):7.3f} ms", flush=True)
    print(f"deep total: split {tot[0]:.3f} ms  nosplit {tot[1]:.3f} ms", flush=True)


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--deep", action="store_true", help="the deeper layers' forwards only")
    a = ap.parse_args()
    from superresolution_for_pdes_amd import hipops as H
    if a.deep:
        return deep(H, a.batch, a.reps)
    dev, hw, n = "cuda", 40, a.batch
    P = n * hw * hw
    for name, c0, c1, cout in LAYERS:
        cin = c0 + c1
        flops = 2.0 * cout * cin * 9 * P
        g = torch.Generator(device=dev).manual_seed(1)
        x = torch.relu(torch.randn(P, cin, device=dev, generator=g))
        x0, x1 = (x[:, :c0], x[:, c0:]) if c1 else (x, None)
        w = torch.randn(cout, cin, 3, 3, device=dev, generator=g) * 0.05
        b = torch.randn(cout, device=dev, generator=g)
        wf, _ = H.pack_conv_weights(w, cin, True, False)
        for t in (x0, x1):
            if t is not None:
                t._srpde_amax = H.amax_of(t)
        gate = aff = None
        if c1:
            gate = (torch.sigmoid(torch.randn(n, c1, device=dev, generator=g)),
                    torch.sigmoid(torch.randn(P, device=dev, generator=g)))
        else:
            aff = (torch.rand(c0, device=dev, generator=g) + 0.5, torch.randn(c0, device=dev, generator=g) * 0.2)
        y = torch.empty(P, cout, device=dev)
        xp = H.split_planes_buffer(P, cin, dev)
        cp = H.cpad32(cout)
        dyp = H.split_planes_buffer(P, cp, dev)
        dyp.normal_()
        dyp._srpde_amax = H.amax_of(torch.randn(16, cp, device=dev))
        dw = torch.empty_like(w)
        res = {"with": [], "plain": [], "plain_nosplit": [], "wgrad": [], "wgrad_x": []}
        xs = H.XSource(x0, x1, aff, gate)
        for _ in range(a.reps):
            stats, _, _ = H.conv_stats_buffer(n, hw, hw, cout, dev, c0, c1, 1)
            res["with"].append(timeit(lambda: H.conv_fwd(x0, x1, wf, b, y, n, hw, hw, cout, 3, 1, 1, False, stats, xp,
                                                         in_affine=aff, x1_gate=gate)))
            res["plain"].append(timeit(lambda: H.conv_fwd(x0, x1, wf, b, y, n, hw, hw, cout, 3, 1, 1, False, stats,
                                                          xp, x1_gate=gate)))
            res["plain_nosplit"].append(timeit(lambda: H.conv_fwd(x0, x1, wf, b, y, n, hw, hw, cout, 3, 1, 1, False,
                                                                  stats, None, x1_gate=gate)))
            res["wgrad"].append(timeit(lambda: H.conv_wgrad_h3p(dyp, xp, dw, n, hw, hw, 3, 1)))
            res["wgrad_x"].append(timeit(lambda: H.conv_wgrad_h3p(dyp, xs, dw, n, hw, hw, 3, 1)))
        line = f"{name:11s}"
        for k, v in res.items():
            if v:
                line += f"  {k} {min(v):7.3f} ms ({flops / min(v) / 1e9 / 838.9:.3f})"
        print(line, flush=True)


if __name__ == "__main__":
    main()
