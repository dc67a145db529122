"""Isolated timing of srpde_bn_bwd_apply_split (the BN backward apply written as dy's h3 split) at the
train step's shapes (batch 1024), as algorithmic GB/s (reads y, da; writes the fp16 hi / lo planes), and of
srpde_bn_bwd_prepare without dgrad partials (its reduce pass over y and da).
usage: python tools/bnb_bench.py [--iters N]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from superresolution_for_pdes_amd import hipops as H  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    n = 1024
    tot_us = tot_prep = 0.0
    for hw, c in ((40, 16), (40, 32), (40, 64), (20, 128), (10, 256), (10, 512)):
        P = n * hw * hw
        y = torch.randn(P, c, device=dev)
        da = torch.randn(P, c, device=dev)
        mean, invstd = y.mean(0), y.var(0).add(1e-5).rsqrt()
        gamma, beta = torch.rand(c, device=dev) + 0.5, torch.randn(c, device=dev) * 0.1
        d1, d2, d3 = (torch.empty(c, device=dev) for _ in range(3))
        m1, m2, word = H.bn_bwd_prepare(y, da, mean, invstd, gamma, beta, d1, d2, d3)
        out = H.split_planes_buffer(P, H.cpad32(c), dev)
        fn = lambda: H.bn_bwd_apply_split(y, da, mean, invstd, gamma, beta, m1, m2, word, out=out)  # noqa: E731
        prep = lambda: H.bn_bwd_prepare(y, da, mean, invstd, gamma, beta, d1, d2, d3)  # noqa: E731
        us, pus = _time(fn, a.iters), _time(prep, a.iters)
        tot_us += us
        tot_prep += pus
        nbytes = P * (8 * c + 4 * H.cpad32(c))
        print(f"P={P:8d} C={c:4d}: apply {us:8.1f} us  {nbytes / us / 1e3:7.1f} GB/s   "
              f"prepare (reduce pass) {pus:8.1f} us  {P * 8 * c / pus / 1e3:7.1f} GB/s")
    print(f"total apply {tot_us:.1f} us, prepare {tot_prep:.1f} us")


def _time(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


if __name__ == "__main__":
    main()
