"""Diagnostic: activation-gradient error of the HIP backward vs the fp64 oracle, stage by stage
(unet_exec.DEBUG_TAPS vs oracle.unet_ref.unet_forward(taps=...)), next to the fp32 oracle's own
error.  Usage: python tools/diag_stages.py [B] [train|eval] [torch seed]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import torch  # noqa: E402

from oracle import unet_ref as U  # noqa: E402
from state import fixture_state_torch  # noqa: E402
from superresolution_for_pdes_amd import unet_exec  # noqa: E402
from superresolution_for_pdes_amd.models import UNet  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
train = not (len(sys.argv) > 2 and sys.argv[2] == "eval")
g = torch.Generator().manual_seed(int(sys.argv[3]) if len(sys.argv) > 3 else 3)
x = torch.randn(B, 3, 40, 40, generator=g)
x[:, 1] = 1.0
t = torch.randn(B, 1, 40, 40, generator=g)

ref = {}
for dt in (torch.float64, torch.float32):
    st = U.clone_state(fixture_state_torch(dt))
    for k in U.trainable_names():
        st[k].requires_grad_(True)
    taps = {}
    out = U.unet_forward(st, x.to(dt), train, taps)
    torch.nn.functional.mse_loss(out, t.to(dt)).backward()
    ref[dt] = {k: v.grad.double() for k, v in taps.items()}

m = UNet()
m.load_state_dict(fixture_state_torch())
m = m.cuda().train(train)
unet_exec.DEBUG_TAPS = {}
torch.nn.functional.mse_loss(m(x.cuda()), t.cuda()).backward()
torch.cuda.synchronize()
ours = unet_exec.DEBUG_TAPS
unet_exec.DEBUG_TAPS = None
print(f"B={B} train={train}")
print(f"{'stage':6s} {'hip_rel':>9s} {'f32_rel':>9s}")
for name in ["o2", "o1", "d1", "u2c", "e1a", "d2", "u3c", "e2a", "d3", "e3a", "b", "b1", "e3", "e2", "e1"]:
    r = ref[torch.float64][name]
    f = ref[torch.float32][name]
    n_, c, h, w = r.shape
    o = ours[name].cpu().double().reshape(n_, h, w, c).permute(0, 3, 1, 2)
    rn = float(r.norm())
    print(f"{name:6s} {float((o - r).norm()) / rn:9.2e} {float((f - r).norm()) / rn:9.2e}")
