"""One 40x40 layer's h5 forward (eval or train variant), --iters launches: the program under rocprofv3 PMC
passes (tools/gpu/h5_pmc.sh).  python tools/h5_one.py [--layer enc1.conv2] [--mode eval|train] [--iters 5]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layer", default="enc1.conv2")
    ap.add_argument("--mode", default="eval", choices=("eval", "train"))
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--h5", type=int, default=1)
    a = ap.parse_args()
    from h5_ab import LAYERS
    from superresolution_for_pdes_amd import hipops as H
    H.set_h5(bool(a.h5))
    name, c0, c1, cout = next(L for L in LAYERS if L[0] == a.layer)
    dev, n, hw = "cuda", a.batch, 40
    P, cin = n * hw * hw, c0 + c1
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(P, cin, device=dev, generator=g)
    x0, x1 = (x[:, :c0], x[:, c0:]) if c1 else (x, None)
    w = torch.randn(cout, cin, 3, 3, device=dev, generator=g) * 0.05
    b = torch.randn(cout, device=dev, generator=g)
    wf, _ = H.pack_conv_weights(w, cin, True, False)
    for t in (x0, x1):
        if t is not None:
            t._srpde_amax = H.amax_of(t)
    y = torch.empty(P, cout, device=dev)
    gate = (torch.sigmoid(torch.randn(n, c1, device=dev, generator=g)),
            torch.sigmoid(torch.randn(P, device=dev, generator=g))) if c1 else None
    if a.mode == "eval":
        ep = (torch.zeros(cout, device=dev), torch.ones(cout, device=dev), torch.ones(cout, device=dev),
              torch.zeros(cout, device=dev), torch.zeros(1, dtype=torch.int32, device=dev))
        fn = lambda: H.conv_fwd(x0, x1, wf, b, y, n, hw, hw, cout, 3, 1, 1, False, None, ep_bn=ep, x1_gate=gate)
    else:
        aff = None if c1 else (torch.rand(c0, device=dev, generator=g) + 0.5,
                               torch.randn(c0, device=dev, generator=g) * 0.2)
        stats, _, _ = H.conv_stats_buffer(n, hw, hw, cout, dev, c0, c1, 1)
        xp = H.split_planes_buffer(P, cin, dev)
        fn = lambda: H.conv_fwd(x0, x1, wf, b, y, n, hw, hw, cout, 3, 1, 1, False, stats, xp, in_affine=aff,
                                x1_gate=gate)
    for _ in range(a.iters):
        fn()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
