"""Diagnostic: per-parameter gradient error of the HIP path vs the fp64 oracle evaluated on the
SAME branch (ReLU masks / max-pool argmaxes of the HIP forward; tests/golden/branch.py), next
to the plain fp64 comparison.  Usage: python tools/diag_branch.py [B] [train|eval] [seed]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import torch  # noqa: E402

from branch import hip_decisions, hip_step  # noqa: E402
from oracle import unet_ref as U  # noqa: E402
from state import fixture_state_torch  # noqa: E402
from superresolution_for_pdes_amd.models import UNet  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
train = not (len(sys.argv) > 2 and sys.argv[2] == "eval")
g = torch.Generator().manual_seed(int(sys.argv[3]) if len(sys.argv) > 3 else 3)
x = torch.randn(B, 3, 40, 40, generator=g)
x[:, 1] = 1.0
t = torch.randn(B, 1, 40, 40, generator=g)
m = UNet()
m.load_state_dict(fixture_state_torch())
m = m.cuda().train(train)
m.flatten_parameters_()
out, grads, dx, S = hip_step(m, x.cuda(), t.cuda())
dec = hip_decisions(m, S)
res = {}
for tag, d in (("branch", dec), ("plain", None)):
    st = U.clone_state(fixture_state_torch(torch.float64))
    for k in U.trainable_names():
        st[k].requires_grad_(True)
    xr = x.double().requires_grad_(True)
    o = U.unet_forward(st, xr, train, decisions=d)
    torch.nn.functional.mse_loss(o, t.double()).backward()
    res[tag] = (o.detach(), {k: st[k].grad for k in U.trainable_names()}, xr.grad)
flips = {k: int((v != (v if k.startswith("pool") else v)).sum()) for k, v in dec.items()}
rel = lambda a, b: float((a.double().cpu() - b).norm() / max(float(b.norm()), 1e-300))  # noqa: E731
print(f"B={B} train={train}")
print(f"output rel err: branch {rel(out.detach(), res['branch'][0]):.2e}  plain {rel(out.detach(), res['plain'][0]):.2e}")
print(f"input grad:     branch {rel(dx, res['branch'][2]):.2e}  plain {rel(dx, res['plain'][2]):.2e}")
print(f"{'param':34s} {'branch':>9s} {'plain':>9s}")
for k in U.trainable_names():
    print(f"{k:34s} {rel(grads[k], res['branch'][1][k]):9.2e} {rel(grads[k], res['plain'][1][k]):9.2e}")
