"""Where the h5 upsampled-input forward differs from h4's and from the materialised upsample (debug aid):
python tools/h5_up_diff.py N"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from superresolution_for_pdes_amd import hipops as H  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
DEV = "cuda"
g = torch.Generator(device=DEV).manual_seed(31)
hw, hl, c0, c1, cout = 40, 20, 128, 64, 64
d = torch.randn(n * hl * hl, c0, device=DEV, generator=g)
e = torch.randn(n * hw * hw, c1, device=DEV, generator=g)
ca = torch.sigmoid(torch.randn(n, c1, device=DEV, generator=g))
w = torch.randn(cout, c0 + c1, 3, 3, device=DEV, generator=g) * 0.05
b = torch.randn(cout, device=DEV, generator=g)
wf, _ = H.pack_conv_weights(w, c0 + c1, True, False)
wg = torch.randn(1, c0, 1, 1, device=DEV, generator=g) * 0.1
bg = torch.randn(1, device=DEV, generator=g)
emean, einv = torch.randn(cout, device=DEV, generator=g) * 0.1, torch.rand(cout, device=DEV, generator=g) + 0.5
ega, ebe = torch.randn(cout, device=DEV, generator=g), torch.randn(cout, device=DEV, generator=g) * 0.1
d._srpde_amax = H.amax_of(d)
e._srpde_amax = H.amax_of(e)
u, sa = H.upsample_gate_fwd(d, n, hl, hl, hw, hw, wg, bg)
P = n * hw * hw
outs = {}
for name, on, x0 in (("h5up", True, H.UpsampledInput(d, n, hl, hl)), ("h4up", False, H.UpsampledInput(d, n, hl, hl)),
                     ("h5mat", True, u)):
    H.set_h5(on)
    ye = torch.empty(P, cout, device=DEV)
    eam = torch.zeros(1, dtype=torch.int32, device=DEV)
    H.conv_fwd(x0, e, wf, b, ye, n, hw, hw, cout, 3, 1, 1, False, None, ep_bn=(emean, einv, ega, ebe, eam),
               x1_gate=(ca, sa))
    torch.cuda.synchronize()
    outs[name] = ye
    print(name, H.last_kernel() if hasattr(H, "last_kernel") else "")
ref = outs["h4up"]
for k in ("h5up", "h5mat"):
    dlt = (outs[k] - ref).abs()
    bad = dlt > 0
    print(f"{k} vs h4up: {int(bad.sum())} differ, max |diff| {float(dlt.max()):.3e}, max rel {float((dlt / ref.abs().clamp_min(1e-3)).max()):.3e}")
    if int(bad.sum()):
        idx = bad.nonzero()
        pix = idx[:, 0]
        rem = pix % (hw * hw)
        print("   rows (y) hit:", sorted(set((rem // hw).tolist()))[:45])
        print("   cols (x) hit:", sorted(set((rem % hw).tolist()))[:45])
        print("   samples:", sorted(set((pix // (hw * hw)).tolist()))[:10])
print("h4up vs h5mat equal:", torch.equal(outs["h4up"], outs["h5mat"]))
