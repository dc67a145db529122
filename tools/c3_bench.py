"""Time the first conv's fused BN-backward + weight gradient (srpde_conv_wgrad_bnb_c3) against the
separate apply (srpde_bn_relu_bwd) + fp32 weight gradient at batch 1024, 40x40, 64 channels.
    python tools/c3_bench.py [--iters 20]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from superresolution_for_pdes_amd import hipops as H  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=1024)
    a, _ = ap.parse_known_args()
    dev = "cuda"
    n, h, C = a.batch, 40, 64
    P = n * h * h
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(P, 4, device=dev, generator=g)
    y = torch.randn(P, C, device=dev, generator=g)
    da = torch.randn(P, C, device=dev, generator=g)
    mean, invstd = y.mean(0), 1.0 / torch.sqrt(y.var(0) + 1e-5)
    gam, bet = torch.ones(C, device=dev), torch.zeros(C, device=dev)
    z = lambda: torch.zeros(C, device=dev)  # noqa: E731
    dy = H.empty(P, C, device=dev)
    dw = torch.empty(C, 3, 3, 3, device=dev)
    dg, db, dc = z(), z(), z()
    m1, m2, _ = H.bn_bwd_prepare(y, da, mean, invstd, gam, bet, dg, db, dc)
    t_apply = timeit(lambda: H.bn_relu_bwd(y, da, mean, invstd, gam, bet, dy, dg, db, dc), a.iters)
    t_wg = timeit(lambda: H.conv_wgrad(dy, x, None, dw, n, h, h), a.iters)
    t_fused = timeit(lambda: H.conv_wgrad_bnb_c3(y, da, mean, invstd, gam, bet, m1, m2, x, dw, n, h, h), a.iters)
    gb = 2 * P * C * 4 / 1e9
    print(f"separate: bn_relu_bwd {t_apply * 1e3:.1f} us + conv_wgrad {t_wg * 1e3:.1f} us; "
          f"fused {t_fused * 1e3:.1f} us ({gb / (t_fused * 1e-3) / 1e3:.2f} TB/s of y + da)")




def first_conv_fwd(iters=20):
    """enc1.conv1 forward (4-float input rows -> 64 channels + BN partials) at batch 1024 (a vector-unit
    kernel for this layer measured 347 us against the fp32 implicit GEMM's 220 us: not kept)."""
    dev = "cuda"
    n, h = 1024, 40
    P = n * h * h
    x = torch.randn(P, 4, device=dev)
    wt = torch.randn(64, 3, 3, 3, device=dev)
    b = torch.randn(64, device=dev)
    wf = H.pack_conv_weights(wt, 4)[0]
    y = H.empty(P, 64, device=dev)
    stats, _, _ = H.conv_stats_buffer(n, h, h, 64, dev, 4)
    t = timeit(lambda: H.conv_fwd(x, None, wf, b, y, n, h, h, 64, 3, 1, 1, False, stats), iters)
    print(f"first conv forward: {t * 1e3:.1f} us ({P * 64 * 4 / (t * 1e-3) / 1e12:.2f} TB/s of y)")


if __name__ == "__main__":
    if "--first-conv" in sys.argv:
        first_conv_fwd()
    else:
        main()
