"""How loose is the rigorous max|dy| bound that sets the dy split's scale (bn.hip
bn_bwd_coef_kernel: |dy_c| <= |gamma_c invstd_c| (max|da| + |m1_c| + sqrt(P-1) |m2_c|))?  Runs one B=1024
train step of the seeded model on synthetic inputs, records every srpde_bn_bwd_apply_split call's bound
word and the true max|dy| of the planes it wrote, and prints bound / actual (log2 = fp16 range bits the
scale leaves unused).  Prints one JSON line.

    python tools/diag_dy_bound.py [--batch 1024]
"""
import argparse
import json
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from superresolution_for_pdes_amd import hipops as H  # noqa: E402
from superresolution_for_pdes_amd.models import UNet, init_weights  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(42)
    m = UNet()
    m.apply(init_weights)
    m = m.to(dev).train()
    g = torch.Generator(device=dev).manual_seed(1234)
    x = torch.randn(a.batch, 3, 40, 40, device=dev, generator=g)
    x[:, 1] = 1.0
    t = torch.randn(a.batch, 1, 40, 40, device=dev, generator=g)
    rec = []
    orig = H.bn_bwd_apply_split

    def spy(y, *args, **kw):
        out = orig(y, *args, **kw)
        rec.append((y.shape[1], out))
        return out

    H.bn_bwd_apply_split = spy
    try:
        out = m(x)
        torch.nn.functional.mse_loss(out, t).backward()
        torch.cuda.synchronize()
    finally:
        H.bn_bwd_apply_split = orig
    rows = []
    for c, planes in rec:
        bound = float(planes._srpde_amax.view(torch.float32).item())
        e = math.floor(math.log2(bound)) + 1
        s = 2.0 ** (15 - e)
        actual = float((planes[0].float() + planes[1].float()).abs().max()) / s
        rows.append({"channels": c, "bound": bound, "actual": actual,
                     "ratio": bound / actual if actual > 0 else None,
                     "unused_bits": math.log2(bound / actual) if actual > 0 else None})
    ratios = [r["ratio"] for r in rows if r["ratio"]]
    print(json.dumps({"batch": a.batch, "calls": rows, "max_ratio": max(ratios), "median_ratio": float(np.median(ratios))}))


if __name__ == "__main__":
    main()
