"""Per-tap timeline of the h5 forward from its timestamp build (conv_h5.hip H5_DBG=16: waves 0 and 4 -- the two
waves of one SIMD -- store s_memtime before and after every tap barrier and around the epilogue of their second
tile).  Prints the mean shader cycles of each segment over the workgroups: 'pre' = from the previous stamp to the
barrier (the tap's work), 'bar' = the wait at the barrier.

    SRPDE_LIB=.../libh5dbg16.so python tools/h5_phase_ts.py [layer] [eval|train]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    from h5_ab import LAYERS
    from superresolution_for_pdes_amd import hipops as H
    name = sys.argv[1] if len(sys.argv) > 1 else "enc1.conv2"
    mode = sys.argv[2] if len(sys.argv) > 2 else "eval"
    _, c0, c1, cout = next(L for L in LAYERS if L[0] == name)
    cin, hw, n, dev = c0 + c1, 40, 1024, "cuda"
    P = n * hw * hw
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(P, cin, device=dev, generator=g)
    x0, x1 = (x[:, :c0], x[:, c0:]) if c1 else (x, None)
    for t in (x0, x1):
        if t is not None:
            t._srpde_amax = H.amax_of(t)
    w = torch.randn(cout, cin, 3, 3, device=dev, generator=g) * 0.05
    wf, _ = H.pack_conv_weights(w, cin, True, False)
    extra = (256 * 512 * 2 + cout - 1) // cout + 1
    ybuf = torch.zeros(P + extra, cout, device=dev)
    y = ybuf[:P]
    gate = (torch.sigmoid(torch.randn(n, c1, device=dev, generator=g)),
            torch.sigmoid(torch.randn(P, device=dev, generator=g))) if c1 else None
    for _ in range(3):
        if mode == "eval":
            ep = (torch.zeros(cout, device=dev), torch.ones(cout, device=dev), torch.ones(cout, device=dev),
                  torch.zeros(cout, device=dev), torch.zeros(1, dtype=torch.int32, device=dev))
            H.conv_fwd(x0, x1, wf, None, y, n, hw, hw, cout, 3, 1, 1, False, None, ep_bn=ep, x1_gate=gate)
        else:
            aff = None if c1 else (torch.rand(c0, device=dev) + 0.5, torch.randn(c0, device=dev) * 0.2)
            stats, _, _ = H.conv_stats_buffer(n, hw, hw, cout, dev, c0, c1, 1)
            xp = H.split_planes_buffer(P, cin, dev)
            H.conv_fwd(x0, x1, wf, None, y, n, hw, hw, cout, 3, 1, 1, False, stats, xp, in_affine=aff, x1_gate=gate)
    torch.cuda.synchronize()
    ts = ybuf[P:].contiguous().view(-1)[:256 * 1024].view(torch.int64).view(256, 8, 64).cpu().numpy()
    k = int(np.median((ts[:, 0] != 0).sum(1)))
    ok = (ts[:, :, :k] != 0).all((1, 2))
    t = ts[ok, :, :k].astype(np.float64)
    t0 = t[:, :, 0].min(1)[:, None, None]
    t = t - t0   # per workgroup, relative to its earliest stamp
    print(f"{name} {mode}: {ok.sum()} workgroups, {k} stamps per wave; mean cycles since the workgroup's first stamp")
    print("  stamp " + " ".join(f"  w{w:d}" for w in range(8)) + "   (even stamps: before a tap barrier, odd: after it)")
    m = t.mean(0)
    for i in range(k):
        print(f"  {i:5d} " + " ".join(f"{m[w, i]:6.0f}" for w in range(8)))
    d = np.diff(t, axis=2).mean(0)
    print("  per-wave time before barriers (work) summed:", " ".join(f"{d[w, 1::2].sum():7.0f}" for w in range(8)))
    print("  per-wave time at barriers summed:           ", " ".join(f"{d[w, 0::2].sum():7.0f}" for w in range(8)))

if __name__ == "__main__":
    main()
