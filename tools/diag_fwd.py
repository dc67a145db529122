"""Diagnostic: per-layer train-mode activation error, HIP vs fp64 oracle, next to fp32 oracle."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import torch, torch.nn.functional as F
from state import fixture_state_torch, fixture_inputs
from oracle import unet_ref as U
from superresolution_for_pdes_amd.models import UNet
from superresolution_for_pdes_amd import unet_exec as X

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
x, t = fixture_inputs(B); x = torch.from_numpy(x)

def ref_acts(dt):
    st = U.clone_state(fixture_state_torch(dt)); xx = x.to(dt); A = {}
    e1 = U.conv_block(st, "enc1", xx, True); A["e1"] = e1
    e2 = U.conv_block(st, "enc2", F.max_pool2d(e1, 2), True); A["e2"] = e2
    e3 = U.conv_block(st, "enc3", F.max_pool2d(e2, 2), True); A["e3"] = e3
    b = F.relu(U._bn_apply(st, "bridge.1", U._conv_apply(st, "bridge.0", e3, 2, 2), True))
    b = F.relu(U._bn_apply(st, "bridge.4", U._conv_apply(st, "bridge.3", b, 2, 2), True)); A["b"] = b
    d3 = U.conv_block(st, "dec3", torch.cat([b, U.attention_gate(st, "att3", e3, b)], 1), True); A["d3"] = d3
    u3 = U.up2(d3); d2 = U.conv_block(st, "dec2", torch.cat([u3, U.attention_gate(st, "att2", e2, u3)], 1), True); A["d2"] = d2
    u2 = U.up2(d2); d1 = U.conv_block(st, "dec1", torch.cat([u2, U.attention_gate(st, "att1", e1, u2)], 1), True); A["d1"] = d1
    yo1 = U._conv_apply(st, "out_conv1", d1, 1); A["yo1"] = yo1
    o1 = F.relu(U._bn_apply(st, "out_bn1", yo1, True)); A["o1"] = o1
    yo2 = U._conv_apply(st, "out_conv2", o1, 1); A["yo2"] = yo2
    o2 = F.relu(U._bn_apply(st, "out_bn2", yo2, True)); A["o2"] = o2
    A["out"] = U._conv_apply(st, "final", o2) + xx[:, 0:1]
    return A

a64, a32 = ref_acts(torch.float64), ref_acts(torch.float32)
m = UNet(); m.load_state_dict(fixture_state_torch()); m = m.cuda().train(); m.flatten_parameters_()
with torch.no_grad():
    out, S = X.unet_forward(m, x.cuda(), True, save=True)
n, h, w = S.shape
def nchw(r, hh):
    return r.reshape(n, hh, hh, -1).permute(0, 3, 1, 2).cpu().double()
mine = {"e1": nchw(S.e1, h), "e2": nchw(S.e2, h // 2), "e3": nchw(S.e3, h // 4), "b": nchw(S.b, h // 4),
        "d3": nchw(S.u3, h // 2), "d2": nchw(S.u2, h), "yo1": nchw(S.out1[2], h), "o1": nchw(S.out2[0], h),
        "yo2": nchw(S.out2[2], h), "o2": nchw(S.o2, h), "out": out.cpu().double()}
for k in mine:
    r = a64[k].double(); f = a32[k].double(); q = mine[k]
    if k in ("d3", "d2"):
        r, f = U.up2(r), U.up2(f)
    rn = float(r.norm())
    print(f"{k:5s} hip {float((q-r).norm())/rn:.2e}  f32 {float((f-r).norm())/rn:.2e}")
for nm, sv in (("out_bn1", S.out1), ("out_bn2", S.out2)):
    print(nm, "mean", sv[3][:4].tolist(), "invstd", sv[4][:4].tolist())
