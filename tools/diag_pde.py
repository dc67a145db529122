"""Diagnose test_pde_dataset_assemble_matches_tensor_expressions: compare the HIP assembly, torch's GPU
expressions and torch's CPU expressions, and print where (element index mod 64) they disagree."""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from superresolution_for_pdes_amd.models import PDEDataset  # noqa: E402


def expr(ucd, ufd, ffd, thd, theta_const):
    um, us = ufd.mean(), ufd.std()
    up = F.interpolate(((ucd - um) / us).unsqueeze(1), size=(40, 40), mode="bilinear", align_corners=True)
    thn = thd if theta_const else (thd - thd.mean()) / thd.std()
    return torch.cat([up, thn.unsqueeze(1), ((ffd - ffd.mean()) / ffd.std()).unsqueeze(1)], dim=1)


for theta_const in (True, False):
    g = torch.Generator().manual_seed(7)
    n = 37
    uc = torch.randn(n, 20, 20, generator=g) * 0.03 + 0.01
    uf = torch.randn(n, 40, 40, generator=g) * 0.03 + 0.01
    ff = torch.randn(n, 40, 40, generator=g) * 5
    th = torch.ones(n, 40, 40) if theta_const else torch.rand(n, 40, 40, generator=g) * 1.5 + 0.5
    ds = PDEDataset({"u_coarse": uc.numpy(), "u_fine": uf.numpy(), "f_fine": ff.numpy(),
                     "theta_fine": th.numpy()}, device="cuda")
    d = torch.device("cuda")
    xg = expr(uc.to(d), uf.to(d), ff.to(d), th.to(d), theta_const).cpu()
    xc = expr(uc, uf, ff, th, theta_const)
    x64 = expr(uc.double(), uf.double(), ff.double(), th.double(), theta_const)
    ours = ds.inputs.cpu()
    for name, a, b in (("hip-torchgpu", ours, xg), ("hip-torchcpu", ours, xc), ("torchgpu-torchcpu", xg, xc), ("hip-fp64", ours.double(), x64),
                          ("torchgpu-fp64", xg.double(), x64), ("torchcpu-fp64", xc.double(), x64)):
        diff = (a - b).abs()
        print(theta_const, name, "max", float(diff.max()), "per-channel", [float(diff[:, c].max()) for c in range(3)])
        bad = (diff[:, 0] > 5e-7).flatten().nonzero().flatten().numpy()
        if bad.size:
            print("   bad count", bad.size, "lane hist", np.bincount(bad % 64, minlength=64).tolist())
            print("   first", bad[:20].tolist())
