"""Phase timing of the h4 forward kernel from its timestamp build (SRPDE_CONV_DBG=256: wave 0 of each
workgroup stores s_memtime at the kernel start, each tile start, after each chunk's 9 taps, after each
between-chunk convert and after the epilogue, into room past the output).  Prints, for one layer, the
mean shader-clock cycles of every phase over the workgroups (first tiles only: 32 stamps per workgroup).

    SRPDE_LIB=.../libsrpde_dbg256.so python tools/h4_phase_ts.py [layer]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

LAYERS = {"enc1.conv2": (64, 64, 40, 1), "dec1.conv2": (64, 64, 40, 1), "enc2.conv2": (128, 128, 20, 1),
          "bridge.3": (512, 512, 10, 2), "dec1.conv1": (192, 64, 40, 1)}


def main():
    from superresolution_for_pdes_amd import hipops as H
    name = sys.argv[1] if len(sys.argv) > 1 else "enc1.conv2"
    cin, cout, hw, dil = LAYERS[name]
    n = 1024
    P = n * hw * hw
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(P, cin, device=dev, generator=g)
    x._srpde_amax = H.amax_of(x)
    w = torch.randn(cout, cin, 3, 3, device=dev, generator=g) * 0.05
    wf, _ = H.pack_conv_weights(w, cin, True, False)
    rows_extra = (256 * 32 * 2 + cout - 1) // cout + 1
    ybuf = torch.zeros(P + rows_extra, cout, device=dev)
    y = ybuf[:P]
    for _ in range(3):
        H.conv_fwd(x, None, wf, None, y, n, hw, hw, cout, 3, dil, 1, False, None)
    torch.cuda.synchronize()
    ts = ybuf[P:].contiguous().view(-1)[:256 * 64].view(torch.int64).view(256, 32).cpu().numpy()
    nz = (ts != 0).sum(1)
    k = int(np.median(nz))
    d = np.diff(ts[:, :k].astype(np.float64), axis=1)
    ok = (ts[:, :k] != 0).all(1)
    d = d[ok]
    print(f"{name}: {ok.sum()} workgroups, {k} stamps each; mean cycles per phase (first tiles):")
    print(" ".join(f"{v:8.0f}" for v in d.mean(0)))
    print("total", float(d.sum(1).mean()))


if __name__ == "__main__":
    main()
