"""Where an h5 forward differs from h4 (debug aid): python tools/h5_diff.py N H C0 C1 COUT [MODE]
MODE: plain (default) | train | eval.  Prints the mismatching (tile, wave row group, pixel block, channel) set."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from superresolution_for_pdes_amd import hipops as H  # noqa: E402

n, h, c0, c1, cout = (int(v) for v in sys.argv[1:6])
mode = sys.argv[6] if len(sys.argv) > 6 else "plain"
DEV = "cuda"
w_ = 40
cin = c0 + c1
g = torch.Generator(device=DEV).manual_seed(17)
P = n * h * w_
x = torch.randn(P, cin, device=DEV, generator=g)
x0, x1 = (x[:, :c0], x[:, c0:]) if c1 else (x, None)
w = torch.randn(cout, cin, 3, 3, device=DEV, generator=g) * 0.05
b = torch.randn(cout, device=DEV, generator=g)
wf, _ = H.pack_conv_weights(w, cin, True, False)
for t in (x0, x1):
    if t is not None:
        t._srpde_amax = H.amax_of(t)
outs = []
for on in (False, True):
    H.set_h5(on)
    for rep in range(3):
        y = torch.full((P, cout), float("nan"), device=DEV)
        H.conv_fwd(x0, x1, wf, b, y, n, h, w_, cout, 3, 1, 1, False, None)
        torch.cuda.synchronize()
        outs.append(y)
ref = outs[0]
for i, y in enumerate(outs):
    bad = (y != ref) | torch.isnan(y)
    nb = int(bad.sum())
    print(f"run {i} (h5={'on' if i >= 3 else 'off'}): {nb} mismatches")
    if nb:
        idx = bad.nonzero()
        pix, ch = idx[:, 0], idx[:, 1]
        tile = pix // 320
        tp = pix % 320
        print("  tiles:", sorted(set(tile.tolist()))[:20])
        print("  wave row group q:", sorted(set((tp // 80).tolist())), " pixel block J:", sorted(set(((tp % 80) // 16).tolist())))
        print("  channels:", sorted(set(ch.tolist()))[:40])
        print("  sample values:", y[pix[:4], ch[:4]].tolist(), ref[pix[:4], ch[:4]].tolist())
