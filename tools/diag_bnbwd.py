"""Diagnostic: one conv+BN+ReLU layer's backward inside the real network, recomputed in fp64
from the executor's OWN saved tensors (conv output y, batch mean / invstd, the incoming
gradient): isolates the BN backward (dy) and the conv dgrad (dx) errors of that layer.
Usage: python tools/diag_bnbwd.py LAYER [B] [train|eval] [seed]   (LAYER e.g. out_conv2, dec3.conv1)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from state import fixture_state_torch  # noqa: E402
from superresolution_for_pdes_amd import unet_exec as X  # noqa: E402
from superresolution_for_pdes_amd.models import UNet  # noqa: E402

layer = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
train = not (len(sys.argv) > 3 and sys.argv[3] == "eval")
g = torch.Generator().manual_seed(int(sys.argv[4]) if len(sys.argv) > 4 else 3)
x = torch.randn(B, 3, 40, 40, generator=g)
x[:, 1] = 1.0
t = torch.randn(B, 1, 40, 40, generator=g)
m = UNet()
m.load_state_dict(fixture_state_torch())
m = m.cuda().train(train)
m.flatten_parameters_()
xd, td = x.cuda(), t.cuda()
with torch.no_grad():
    out, S = X.unet_forward(m, xd, train, save=True)
    dout = (2.0 / out.numel()) * (out - td)
    layout = m._flat_layout()
    flat = torch.empty(layout[-1][2] + layout[-1][3], device="cuda")
    views = {p: flat[o:o + n].view_as(p) for _, p, o, n in layout}
    X.DEBUG_TAPS = {}
    X.unet_backward(m, S, dout, views)
    torch.cuda.synchronize()
taps = X.DEBUG_TAPS
# locate the layer's saved tuple and its BN
mods = dict(m.named_modules())
conv = mods[layer]
bn_name = {"out_conv1": "out_bn1", "out_conv2": "out_bn2", "bridge.0": "bridge.1", "bridge.3": "bridge.4"}.get(
    layer, layer.replace("conv", "bn"))
bn = mods[bn_name]
saved_of = {"out_conv1": S.out1, "out_conv2": S.out2, "bridge.0": S.br1, "bridge.3": S.br2}
if layer not in saved_of:
    blk, which = layer.split(".")
    saved_of[layer] = getattr(S, blk)[0 if which == "conv1" else 1]
x0, x1, y, mean, invstd, xp, tr = saved_of[layer]
dy_ours = taps["dy:" + layer].double()
P, C = y.shape
# the incoming gradient da: recover it from the next stage tap names is layer-specific; recompute
# dy in fp64 from OUR da, which the executor keeps nowhere -> use the bn_relu_bwd contract: the
# BN backward's input is the tap of the previous stage
prev = {"out_conv2": "o2", "out_conv1": "o1", "dec1.conv2": "d1"}.get(layer)
if prev is None:
    print("no incoming-gradient tap for", layer)
    sys.exit(0)
da = taps[prev].double()
yd, mu, iv = y.double(), mean.double(), invstd.double()
ga, be = bn.weight.detach().double(), bn.bias.detach().double()
xh = (yd - mu) * iv
dz = da * ((xh * ga + be) > 0)
if tr:
    m1, m2 = dz.mean(0), (dz * xh).mean(0)
    dy_ref = ga * iv * (dz - m1 - xh * m2)
else:
    dy_ref = ga * iv * dz
rel = lambda a, b: float((a - b).norm() / b.norm())  # noqa: E731
print(f"{layer}: P={P} C={C} train={tr}")
print(f"  BN bwd dy rel err (ours vs fp64 from our inputs) {rel(dy_ours, dy_ref):.3e}")
print(f"  cancellation |dz| / |dz - m1 - xh m2| = {float(dz.norm() / (dy_ref / (ga * iv)).norm()):.3e}")
# dgrad from our dy, fp64, vs our dx tap
nxt = {"out_conv2": "o1", "out_conv1": "d1"}.get(layer)
if nxt is not None:
    n_, h_, w_ = S.shape
    cin = conv.in_channels
    dyn = dy_ours.reshape(n_, h_, w_, C).permute(0, 3, 1, 2)
    dx_ref = torch.nn.grad.conv2d_input((n_, cin, h_, w_), conv.weight.detach().double(), dyn, padding=1)
    dx = taps[nxt].double().reshape(n_, h_, w_, cin).permute(0, 3, 1, 2)
    print(f"  dgrad rel err (ours vs fp64 from our dy) {rel(dx, dx_ref):.3e}")


# forward side: our saved activations vs the fp64 oracle's forward (same weights and inputs)
from oracle import unet_ref as U  # noqa: E402
st = U.clone_state(fixture_state_torch(torch.float64))
taps64 = {}
for k in U.trainable_names():
    st[k].requires_grad_(True)
U.unet_forward(st, x.double(), train, taps64)
n_, h_, w_ = S.shape
def nhwc(t, c):  # noqa: E302
    return t.detach().double().cpu().reshape(n_, h_, w_, c).permute(0, 3, 1, 2)
if layer in ("out_conv2", "out_conv1"):
    src = "o1" if layer == "out_conv2" else "d1"
    a_ref = taps64[src].detach()
    a_our = nhwc(x0, a_ref.shape[1])
    print(f"  fwd input activation ({src}) rel err {rel(a_our, a_ref):.3e}")
    y_ref = F.conv2d(a_ref, conv.weight.detach().double().cpu(), conv.bias.detach().double().cpu(), padding=1)
    y_our = nhwc(y, C)
    print(f"  fwd conv output rel err {rel(y_our, y_ref):.3e}; from our input in fp64: "
          f"{rel(y_our, F.conv2d(a_our, conv.weight.detach().double().cpu(), conv.bias.detach().double().cpu(), padding=1)):.3e}")
    mref = y_ref.mean(dim=(0, 2, 3))
    vref = y_ref.var(dim=(0, 2, 3), unbiased=False)
    print(f"  batch mean rel err {rel(mean.double().cpu(), mref):.3e}  invstd rel err "
          f"{rel(invstd.double().cpu(), 1 / torch.sqrt(vref + 1e-5)):.3e}")

# backward side against the oracle's own activation gradients
out64 = U.unet_forward(U.clone_state(fixture_state_torch(torch.float64)), x.double(), train, None)
st2 = U.clone_state(fixture_state_torch(torch.float64))
for k in U.trainable_names():
    st2[k].requires_grad_(True)
taps_b = {}
o64 = U.unet_forward(st2, x.double(), train, taps_b)
F.mse_loss(o64, t.double()).backward()
print(f"  output rel err {rel(out.detach().double().cpu().reshape(o64.shape), o64.detach()):.3e}")
for nm in ("o2", "o1", "d1"):
    r = taps_b[nm].grad
    c_ = r.shape[1]
    print(f"  grad {nm}: direct-executor rel err {rel(nhwc(taps[nm], c_), r):.3e}")
# the same through autograd (UNetFunction.backward: wgrad side stream)
m2 = UNet()
m2.load_state_dict(fixture_state_torch())
m2 = m2.cuda().train(train)
X.DEBUG_TAPS = {}
F.mse_loss(m2(xd), td).backward()
torch.cuda.synchronize()
for nm in ("o2", "o1", "d1"):
    r = taps_b[nm].grad
    print(f"  grad {nm}: autograd-path rel err {rel(nhwc(X.DEBUG_TAPS[nm], r.shape[1]), r):.3e}")

X.DEBUG_TAPS = None
# fp64 chain from the ORACLE's forward values: do2 -> dy2 -> do1
if layer == "out_conv2":
    o1r = taps_b["o1"].detach()
    y2r = F.conv2d(o1r, conv.weight.detach().double().cpu(), conv.bias.detach().double().cpu(), padding=1)
    mu_r = y2r.mean(dim=(0, 2, 3), keepdim=True)
    iv_r = 1 / torch.sqrt(y2r.var(dim=(0, 2, 3), unbiased=False, keepdim=True) + 1e-5)
    gr = bn.weight.detach().double().cpu().view(1, -1, 1, 1)
    br = bn.bias.detach().double().cpu().view(1, -1, 1, 1)
    xhr = (y2r - mu_r) * iv_r
    dzr = taps_b["o2"].grad * ((xhr * gr + br) > 0)
    dyr = gr * iv_r * (dzr - dzr.mean(dim=(0, 2, 3), keepdim=True) - xhr * (dzr * xhr).mean(dim=(0, 2, 3), keepdim=True))
    do1r = torch.nn.grad.conv2d_input(o1r.shape, conv.weight.detach().double().cpu(), dyr, padding=1)
    print(f"  fp64 chain from oracle values: do1 vs oracle autograd {rel(do1r, taps_b['o1'].grad):.3e}")
    print(f"  our dy vs fp64 chain dy {rel(nhwc(dy_ours, C), dyr):.3e}")
    mk_o = ((nhwc(y, C) - nhwc(mean.view(1, -1).expand(P, -1), C)) * nhwc(invstd.view(1, -1).expand(P, -1), C) * gr + br) > 0
    print(f"  mask flips {int((mk_o != ((xhr * gr + br) > 0)).sum())} of {mk_o.numel()}")
    print(f"  |xh*g+b| min {float((xhr * gr + br).abs().min()):.3e}")
