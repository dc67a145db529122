"""Isolated timing of the HBM-bound BatchNorm kernels and the upsample backward at the training
step's shapes (batch 1024), reported as algorithmic GB/s.  The train step runs these beside the
weight-gradient side stream; here each runs alone.
usage: python tools/pw_bench.py [--iters N]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from superresolution_for_pdes_amd import hipops as H  # noqa: E402

D = torch.device("cuda", 0)


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    tag = "isolated"
    B = 1024
    for hw, c in ((40, 64), (40, 32), (20, 128), (10, 512)):
        P = B * hw * hw
        y = torch.randn(P, c, device=D)
        da = torch.randn(P, c, device=D)
        mean, invstd = torch.zeros(c, device=D), torch.ones(c, device=D)
        gam, bet = torch.ones(c, device=D), torch.zeros(c, device=D)
        out = H.empty(P, c, device=D)
        amax = torch.zeros(1, dtype=torch.int32, device=D)
        t = timed(lambda: H.bn_relu_fwd(y, mean, invstd, gam, bet, out, amax=amax), a.iters)
        print(f"{tag} bn_relu_fwd P={P} C={c}: {t:8.1f} us  {8 * P * c / t / 1e3:7.0f} GB/s")
        dg, db, dbias = (torch.empty(c, device=D) for _ in range(3))
        t = timed(lambda: H.bn_relu_bwd(y, da, mean, invstd, gam, bet, out, dg, db, dbias, amax=amax), a.iters)
        # reduce pass reads y, da; apply pass reads y, da and writes dy
        print(f"{tag} bn_relu_bwd P={P} C={c}: {t:8.1f} us  {20 * P * c / t / 1e3:7.0f} GB/s")
        del y, da, out
    for h, c in ((20, 128), (10, 256)):
        ho = 2 * h
        dout = torch.randn(B * ho * ho, c, device=D)
        dx = H.empty(B * h * h, c, device=D)
        dsa, wg = torch.randn(B * ho * ho, device=D), torch.randn(c, device=D)
        t = timed(lambda: H.upsample_bwd(dout, dx, B, h, h, ho, ho, False, gate=(dsa, wg)), a.iters)
        nb = 4 * (B * ho * ho * (c + 1) + B * h * h * c)
        print(f"upsample_bwd_gated {h}->{ho} C={c}: {t:8.1f} us  {nb / t / 1e3:7.0f} GB/s")


if __name__ == "__main__":
    main()
