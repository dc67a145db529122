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
    ap.add_argument("--seeds", type=int, default=5, help="test fields (np.random seeds 0..seeds-1)")
    ap.add_argument("--save", default=None,
                    help="dir: best weights (model_state_dict, fp32) + seed-0 cascade outputs, for the CPU "
                         "cross-check against the reference (tests/golden/crosscheck_trained_cascade.py)")
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

    from superresolution_for_pdes_amd.resolution_comparison_enhanced import compare_resolutions
    per_seed = []
    for seed in range(args.seeds):
        np.random.seed(seed)
        data = RC.solve_multi_resolution(n_coarse=40, resolutions=[80, 160, 320, 640])
        sols, met = compare_resolutions(model, data)
        per_seed.append({"seed": seed, "k1": data["k1"], "k2": data["k2"],
                         "metrics": {m: {str(r): v for r, v in d.items()} for m, d in met.items()}})
        if seed == 0 and args.save:
            os.makedirs(args.save, exist_ok=True)
            torch.save({k: v.detach().cpu() for k, v in model.state_dict().items()},
                       os.path.join(args.save, "e2e_best_weights.pt"))
            np.savez_compressed(os.path.join(args.save, "e2e_seed0_cascade.npz"),
                                **{f"ml{r}": sols["ml"][r].astype(np.float32) for r in (80, 160, 320, 640)})
    table = {}
    for res in (80, 160, 320, 640):
        table[res] = {m: {"mae_mean": float(np.mean([ps["metrics"][m][str(res)]["mae"] for ps in per_seed])),
                          "rmse_mean": float(np.mean([ps["metrics"][m][str(res)]["rmse"] for ps in per_seed]))}
                      for m in per_seed[0]["metrics"]}
        table[res]["ml_over_best_interp_mae"] = table[res]["ml"]["mae_mean"] / min(
            table[res][m]["mae_mean"] for m in table[res] if m != "ml")
    rec = {"what": "device data-gen + training (reference config) + resolution comparison",
           "samples": list(args.n), "epochs_run": len(hist["train_loss"]), "best_epoch": hist["best_epoch"],
           "best_val_loss": hist["best_val_loss"], "final_train_loss": hist["train_loss"][-1],
           "wall_s_generate_and_train": round(train_s, 1),
           "s_per_epoch": round(train_s / max(1, len(hist["train_loss"])), 3),
           "resolution_comparison_mean_over_seeds": {str(k): v for k, v in table.items()},
           "per_seed": per_seed}
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
