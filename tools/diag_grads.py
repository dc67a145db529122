"""Diagnostic: per-parameter gradient error of the HIP U-Net vs the fp64 oracle, next to
the fp32 oracle's own error (same inputs).  Usage: python tools/diag_grads.py [B] [train|eval] [torch seed]"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden"))
import numpy as np, torch
from state import fixture_state_torch, fixture_inputs
from oracle import unet_ref as U
from superresolution_for_pdes_amd.models import UNet

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
train = not (len(sys.argv) > 2 and sys.argv[2] == "eval")
if len(sys.argv) > 3:   # torch.randn inputs as the GPU tests draw them: seed
    g = torch.Generator().manual_seed(int(sys.argv[3]))
    x = torch.randn(B, 3, 40, 40, generator=g); x[:, 1] = 1.0
    t = torch.randn(B, 1, 40, 40, generator=g)
else:
    x, t = fixture_inputs(B)
    x, t = torch.from_numpy(x), torch.from_numpy(t)
_, _, g64, _ = U.forward_with_grads(fixture_state_torch(torch.float64), x.double(), t.double(), train)
_, _, g32, _ = U.forward_with_grads(fixture_state_torch(torch.float32), x, t, train)
m = UNet(); m.load_state_dict(fixture_state_torch()); m = m.cuda().train(train)
out = m(x.cuda()); torch.nn.functional.mse_loss(out, t.cuda()).backward()
P = dict(m.named_parameters())
print(f"B={B} train={train}")
print(f"{'param':34s} {'hip_rel':>9s} {'f32_rel':>9s} {'hip_nrm':>10s} {'f32_nrm':>10s}")
for n in g64:
    a = P[n].grad.detach().cpu().double().reshape(-1); r = g64[n].reshape(-1); f = g32[n].double().reshape(-1)
    rn = max(float(r.norm()), 1e-30)
    print(f"{n:34s} {float((a-r).norm())/rn:9.2e} {float((f-r).norm())/rn:9.2e} {float(a.norm())/rn-1:10.2e} {float(f.norm())/rn-1:10.2e}")
