"""Interpolation baselines of the cascade evaluation (config #5's accuracy table) on MI355X.

Reference: src/resolution_comparison_enhanced.py -- ``bilinear_multi_level_upscale`` :19-41,
``cubic_multi_level_upscale`` :43-65, and the direct (one-step) bilinear / bicubic resizes plus
the MAE / RMSE of every method against the ground truth in ``main`` :355-415.  These are the
"Bilinear" / "Cubic" rows the reference's published numbers compare the ML cascade against
(README.md:139-144).  Semantics kept: the 40x40 ground truth is cast to fp32
(``torch.from_numpy(u).float()``) and resized with align_corners=True, repeatedly by 2x
(multi-level) or once to the target (direct); results are fp32 numpy fields.  The resizes run
on the HIP kernels (srpde_upsample_bilinear_fwd, srpde_resize_bicubic_ac); plots are out of
scope, the metrics are returned / written as JSON instead.
"""
from __future__ import annotations

import argparse
import json
import os
from typing import Dict, List

import numpy as np
import torch

from . import hipops as H
from .resolution_comparison import ml_multi_level_upscale, solve_multi_resolution


def _resize(u: torch.Tensor, size: int, mode: str) -> torch.Tensor:
    """[h, w] fp32 device field -> [size, size] (align_corners=True)."""
    h, w = u.shape
    if mode == "bilinear":
        out = H.upsample_fwd(u.contiguous().view(h * w, 1), 1, h, w, size, size)
        return out.view(size, size)
    if mode == "bicubic":
        return H.resize_bicubic(u.contiguous().view(1, h, w), size, size)[0]
    raise ValueError(mode)


def _start(data: dict, device) -> torch.Tensor:
    u = data["u"][40]
    u = u if isinstance(u, torch.Tensor) else torch.from_numpy(np.asarray(u))
    return u.to(device=device, dtype=torch.float64).float()    # .float() of the fp64 field, as :33


def _multi_level(data: dict, target_resolution: int, mode: str, device="cuda") -> np.ndarray:
    cur, res = _start(data, device), 40
    while res < target_resolution:
        res *= 2
        cur = _resize(cur, res, mode)
    return cur.cpu().numpy()


def bilinear_multi_level_upscale(data: dict, target_resolution: int, device="cuda") -> np.ndarray:
    """resolution_comparison_enhanced.py:19-41: repeated 2x bilinear (align_corners) from 40^2."""
    return _multi_level(data, target_resolution, "bilinear", device)


def cubic_multi_level_upscale(data: dict, target_resolution: int, device="cuda") -> np.ndarray:
    """resolution_comparison_enhanced.py:43-65: repeated 2x bicubic (align_corners) from 40^2."""
    return _multi_level(data, target_resolution, "bicubic", device)


def direct_upscale(data: dict, target_resolution: int, mode: str, device="cuda") -> np.ndarray:
    """resolution_comparison_enhanced.py:371-392: one resize of the 40^2 field to the target."""
    return _resize(_start(data, device), target_resolution, mode).cpu().numpy()


def _metrics(pred, gt) -> Dict[str, float]:
    e = np.asarray(pred, np.float64) - np.asarray(gt, np.float64)
    return {"mae": float(np.mean(np.abs(e))), "rmse": float(np.sqrt(np.mean(e ** 2)))}


def compare_resolutions(model, data: dict, resolutions: List[int] = (80, 160, 320, 640), device="cuda"):
    """The method comparison of main() (:355-415) without the plots: per target resolution the
    ML cascade, multi-level and direct bilinear / bicubic fields and their MAE / RMSE against the
    ground truth ``data['u'][res]``.  Returns (solutions, metrics) dicts keyed by method then res."""
    sols = {k: {} for k in ("ml", "bilinear_multi", "bilinear_direct", "cubic_multi", "cubic_direct")}
    for res in resolutions:
        sols["ml"][res] = ml_multi_level_upscale(model, data, res, device)
        sols["bilinear_multi"][res] = bilinear_multi_level_upscale(data, res, device)
        sols["bilinear_direct"][res] = direct_upscale(data, res, "bilinear", device)
        sols["cubic_multi"][res] = cubic_multi_level_upscale(data, res, device)
        sols["cubic_direct"][res] = direct_upscale(data, res, "bicubic", device)
    metrics = {k: {res: _metrics(v[res], data["u"][res]) for res in resolutions} for k, v in sols.items()}
    return sols, metrics


def main(argv=None):
    """CLI of the reference (:319-422, ``--model_path``): metrics JSON next to the checkpoint."""
    from .compare_methods import load_model
    ap = argparse.ArgumentParser()
    ap.add_argument("--model_path", type=str, required=True)
    ap.add_argument("--seed", type=int, default=None, help="np.random seed of the test field (reference: unseeded)")
    args = ap.parse_args(argv)
    if args.seed is not None:
        np.random.seed(args.seed)
    model = load_model(args.model_path, "cuda")
    model.eval()
    out_dir = os.path.join(os.path.dirname(os.path.abspath(args.model_path)), "resolution_comparison_enhanced_results")
    os.makedirs(out_dir, exist_ok=True)
    data = solve_multi_resolution(n_coarse=40, resolutions=[80, 160, 320, 640])
    _, metrics = compare_resolutions(model, data)
    for res in (80, 160, 320, 640):
        print(f"\nResults for {res}x{res}:")
        for name, label in (("ml", "ML Multi-level"), ("bilinear_multi", "Bilinear Multi-level"),
                            ("bilinear_direct", "Direct Bilinear"), ("cubic_multi", "Cubic Multi-level"),
                            ("cubic_direct", "Direct Cubic")):
            mt = metrics[name][res]
            print(f"{label} - MAE: {mt['mae']:.6f}, RMSE: {mt['rmse']:.6f}")
    with open(os.path.join(out_dir, "metrics.json"), "w") as f:
        json.dump({k: {str(r): v for r, v in d.items()} for k, d in metrics.items()}, f, indent=2)
    return metrics


if __name__ == "__main__":
    main()
