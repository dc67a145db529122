"""End-to-end run of the drop-in on one MI355X: generate the reference's training set on the
device (config #3), train with the reference's config (train_enhanced.main), then the
reference's resolution comparison (src/resolution_comparison.py:371-430: 40 -> 80/160/320/640
cascade vs the ground-truth solve, against direct bilinear) with the trained model.

    python tools/e2e_accuracy.py [--epochs 100] [--out /tmp/srpde_e2e]
Prints one JSON line (timings + the MAE/RMSE table the reference's README reports).
"""
import argparse
import glob
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=100)
    ap.add_argument("--n", type=int, nargs=2, default=(1000, 1000))
    ap.add_argument("--out", default="/tmp/srpde_e2e")   # checkpoints stay out of gpurun_out/
    args = ap.parse_args()
    from superresolution_for_pdes_amd import train_enhanced as T
    from superresolution_for_pdes_amd import resolution_comparison as RC
    from superresolution_for_pdes_amd.compare_methods import load_model

    torch.cuda.synchronize()
    t0 = time.perf_counter()
    hist = T.main(["--generate", str(args.n[0]), str(args.n[1]), "--epochs", str(args.epochs),
                   "--results", args.out])
    torch.cuda.synchronize()
    train_s = time.perf_counter() - t0
    best = sorted(glob.glob(os.path.join(args.out, "*", "best_model.pth")))[-1]
    model = load_model(best, "cuda")
    model.eval()

    np.random.seed(0)
    data = RC.solve_multi_resolution(n_coarse=40, resolutions=[80, 160, 320, 640])
    table = {}
    for res in (80, 160, 320, 640):
        ml = RC.ml_multi_level_upscale(model, data, res, "cuda")
        bl = F.interpolate(torch.from_numpy(data["u"][40]).float()[None, None], size=(res, res), mode="bilinear",
                           align_corners=True).squeeze().numpy()
        gt = data["u"][res]
        table[res] = {"ml": RC.cascade_metrics(ml, gt), "bilinear": RC.cascade_metrics(bl, gt)}
    rec = {"what": "device data-gen + training (reference config) + resolution comparison",
           "samples": list(args.n), "epochs_run": len(hist["train_loss"]), "best_epoch": hist["best_epoch"],
           "best_val_loss": hist["best_val_loss"], "final_train_loss": hist["train_loss"][-1],
           "wall_s_generate_and_train": round(train_s, 1),
           "s_per_epoch": round(train_s / max(1, len(hist["train_loss"])), 3),
           "resolution_comparison": {str(k): v for k, v in table.items()}}
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
