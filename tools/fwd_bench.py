"""The B=1024 40x40 U-Net forward alone (north_star's roofline target), for rocprofv3 kernel summaries.

    python tools/fwd_bench.py --mode eval|train [--iters N] [--batch B]

Same model / inputs as bench.py (seed-42 init, synthetic x), ``--iters`` forwards after 3 warm-ups,
HIP events around them; prints one JSON line (ms per forward, HBM and MFMA fractions as bench.py's
roofline.forward).  Under ``rocprofv3 --kernel-trace --stats`` the kernel table divided by --iters
(+3 warm-ups) is the forward's per-kernel composition (profiles/*_fwd_*_kernel_stats.csv)."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=("eval", "train"), default="eval")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args()
    import bench
    from superresolution_for_pdes_amd.models import UNet, init_weights
    dev = torch.device("cuda", 0)
    torch.manual_seed(42)
    model = UNet()
    model.apply(init_weights)
    model = model.to(dev)
    g = torch.Generator(device=dev).manual_seed(1234)
    x = torch.randn(a.batch, 3, 40, 40, device=dev, generator=g)
    x[:, 1] = 1.0
    ms = bench.time_forward(model, x, a.mode == "train", reps=a.iters, warm=3)
    t = ms * 1e-3
    B = a.batch
    print(json.dumps({"mode": a.mode, "batch": B, "iters": a.iters, "ms": round(ms, 4),
                      "hbm_frac": round(bench.FWD_BYTES_PER_SAMPLE * B / t / bench.HBM_PEAK, 4),
                      "mfma_frac": round(bench.FWD_FLOP_PER_SAMPLE * B / t / 838.9e12, 4)}))


if __name__ == "__main__":
    main()
