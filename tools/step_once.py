"""bench.py's training step (B=1024 40x40 U-Net, forward + MSE + backward + clip + AdamW), --steps times after one
warm-up, nothing printed: the program the roofline's PMC passes run (bench.py measure_step_traffic).
    python tools/step_once.py [--steps 2] [--batch 1024]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args()
    from superresolution_for_pdes_amd.models import UNet, init_weights
    from superresolution_for_pdes_amd.functional import mse_loss
    from superresolution_for_pdes_amd.optim import FusedAdamW
    dev = torch.device("cuda", 0)
    torch.manual_seed(42)
    model = UNet()
    model.apply(init_weights)
    model = model.to(dev).train()
    model.flatten_parameters_()
    opt = FusedAdamW(model.parameters(), lr=2e-4, weight_decay=1e-4, max_grad_norm=1.0)
    g = torch.Generator(device=dev).manual_seed(1234)
    x = torch.randn(a.batch, 3, 40, 40, device=dev, generator=g)
    x[:, 1] = 1.0
    tgt = torch.randn(a.batch, 1, 40, 40, device=dev, generator=g)
    for _ in range(1 + a.steps):
        for p in model.parameters():
            p.grad = None
        loss = mse_loss(model(x), tgt)
        loss.backward()
        opt.step()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
