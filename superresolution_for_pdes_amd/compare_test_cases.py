"""Evaluation report of reference src/compare_test_cases.py, on the device.

Same test sets, draw order and metrics as the reference; the plots (matplotlib / seaborn) are
out of scope.  Differences in mechanism, not in result:

* the ground truth comes from the batched on-device CG (``poisson.solve_batched``) instead of one
  ``spsolve`` per sample (compare_test_cases.py:38-68);
* the model runs on the whole set in batches (eval mode: BatchNorm uses running statistics, so a
  sample's prediction does not depend on its batch), instead of one sample at a time (:113-117);
* the bilinear baseline is the HIP resize of the raw coarse field in fp32 (:120-125) and the
  per-sample MAE / RMSE are fp64 reductions on the device of the same fp32-vs-fp64 differences
  numpy forms (:130-135).

``main`` writes ``comprehensive_test_results.json`` next to the model (:629-674).
"""
from __future__ import annotations

import argparse
import json
from pathlib import Path

import numpy as np
import torch

from . import poisson as P
from .compare_methods import load_model
from .data_generation import PoissonSolver
from .models import PDEDataset, upsample_bilinear


def generate_test_data(k_range: tuple, n_samples: int = 10, label: str = "test", constant_theta: bool = True,
                       save_dir: str | None = None, device: str = "cuda") -> dict:
    """compare_test_cases.py:12-79.  ``constant_theta``: theta = 1 (the solves of
    ``generate_dataset`` already are theta = 1, so re-solving reproduces them); otherwise one
    U(0.5, 2) theta field per sample, drawn in sample order after the k draws, coarse theta =
    theta_fine[::2, ::2], and both grids re-solved.  ``save_dir``: also np.savez the set as
    ``{label}_dataset.npz`` there (the reference always saves under data/)."""
    solver = PoissonSolver(device=device)
    data = solver.generate_dataset(n_samples=n_samples, k_range=k_range)
    nf = solver.n_fine
    if constant_theta:
        data["theta_fine"] = np.ones_like(data["theta_fine"])
        data["theta_coarse"] = np.ones_like(data["theta_coarse"])
    else:
        th_f = np.empty((n_samples, nf, nf))
        for i in range(n_samples):        # same draw order as the reference loop
            th_f[i] = np.random.uniform(0.5, 2.0, size=(nf, nf))
        th_c = np.ascontiguousarray(th_f[:, ::2, ::2])
        data["theta_fine"], data["theta_coarse"] = th_f, th_c
        data["u_fine"] = P.solve_batched(data["f_fine"], th_f, device=device).cpu().numpy()
        data["u_coarse"] = P.solve_batched(data["f_coarse"], th_c, device=device).cpu().numpy()
    if save_dir is not None:
        path = Path(save_dir)
        path.mkdir(parents=True, exist_ok=True)
        np.savez(path / f"{label}_dataset.npz", **data)
    return data


def _predict(model, ds: PDEDataset, batch: int) -> torch.Tensor:
    outs = []
    with torch.no_grad():
        for i in range(0, len(ds), batch):
            outs.append(model(ds.inputs[i:i + batch]))
    return ds.denormalize(torch.cat(outs))[:, 0]


def evaluate_dataset(data: dict, model, device: str = "cuda", label: str = "test", batch: int = 256,
                     theta_range: bool = False):
    """compare_test_cases.py:81-247 (metrics only) -> (per-sample metrics, averages).
    ``theta_range``: add each sample's [min, max] theta, as the training-like report does (:305)."""
    model.eval()
    ds = PDEDataset(data, device=device)
    ml = _predict(model, ds, batch).double()
    nf = ds.u_fine.shape[-1]
    uc = torch.as_tensor(np.asarray(data["u_coarse"]), dtype=torch.float32).to(device).unsqueeze(1)
    bl = upsample_bilinear(uc.contiguous(), nf, nf)[:, 0].double()
    fine = torch.as_tensor(np.asarray(data["u_fine"]), dtype=torch.float64).to(device)

    def mae_rmse(x):
        d = x - fine
        return d.abs().mean((1, 2)), d.pow(2).mean((1, 2)).sqrt()

    bmae, brmse = (t.cpu().numpy() for t in mae_rmse(bl))
    mmae, mrmse = (t.cpu().numpy() for t in mae_rmse(ml))
    th = np.asarray(data["theta_fine"])
    metrics = []
    for i in range(len(ds)):
        m = {"k1": float(data["k1"][i]), "k2": float(data["k2"][i]),
             "bilinear_mae": float(bmae[i]), "bilinear_rmse": float(brmse[i]),
             "ml_mae": float(mmae[i]), "ml_rmse": float(mrmse[i])}
        if theta_range:
            m["theta_range"] = [float(th[i].min()), float(th[i].max())]
        metrics.append(m)
    avg = {k: float(np.mean([m[k[4:]] for m in metrics]))
           for k in ("avg_bilinear_mae", "avg_bilinear_rmse", "avg_ml_mae", "avg_ml_rmse")}
    return metrics, avg


def evaluate_training_like_cases(model, device: str = "cuda", n_samples: int = 25, batch: int = 256):
    """compare_test_cases.py:249-413: the training generator's own process, k ~ U(0.5, 5)."""
    solver = PoissonSolver(n_coarse=20, n_fine=40, device=device)
    data = solver.generate_dataset(n_samples=n_samples, k_range=(0.5, 5.0))
    return evaluate_dataset(data, model, device, "training_like", batch, theta_range=True)


def run_report(model, n_samples: int = 16, device: str = "cuda", save_dir: str | None = None) -> dict:
    """The five evaluations of main() (compare_test_cases.py:629-670), in the reference's order."""
    tr, tr_avg = evaluate_training_like_cases(model, device, n_samples)
    out = {"training_like": {"individual_metrics": tr, "average_metrics": tr_avg}}
    for key, const in (("constant_theta", True), ("varying_theta", False)):
        out[key] = {}
        for part, kr in (("in_sample", (1.0, 6.0)), ("out_of_sample", (6.0, 8.0))):
            tag = "const_theta" if const else "var_theta"
            data = generate_test_data(kr, n_samples, f"{part}_{tag}", const, save_dir, device)
            m, avg = evaluate_dataset(data, model, device, part)
            out[key][part] = {"individual_metrics": m, "average_metrics": avg}
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description="Compare in-sample and out-of-sample test cases")
    ap.add_argument("--model_path", type=str, required=True, help="Path to the model file")
    ap.add_argument("--n_samples", type=int, default=16, help="Number of samples for each test")
    args = ap.parse_args(argv)
    model_path = Path(args.model_path)
    if not model_path.exists():
        raise FileNotFoundError(f"Model not found at path: {model_path}")
    model = load_model(model_path, "cuda")
    model.eval()
    results = run_report(model, args.n_samples, "cuda", save_dir="data")
    with open(model_path.parent / "comprehensive_test_results.json", "w") as f:
        json.dump(results, f, indent=4)
    return results


if __name__ == "__main__":
    main()
