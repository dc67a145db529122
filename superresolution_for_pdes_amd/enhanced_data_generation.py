"""Drop-in for reference ``src/enhanced_data_generation.py`` with batched on-device solves.

``EnhancedPoissonSolver(n_coarse, n_fine, n_superfine)`` (enhanced_data_generation.py:11-244):
subdomain samples solve on the super-fine grid (80^2), crop a random n_fine window
(start in [0, n_superfine - n_fine)) and stride by 2 for the coarse grid.  The random draws
(k1, k2, start_x, start_y per sample, global np.random) keep the reference's order, so a
seeded run reproduces the reference's dataset; all super-fine solves run as one batch.
"""
from __future__ import annotations

from typing import Dict, Tuple

import numpy as np
import torch

from . import poisson as P
from .data_generation import PoissonSolver, gather_fields, resolve_shard, shard_range, to_numpy


class EnhancedPoissonSolver(PoissonSolver):
    def __init__(self, n_coarse: int = 20, n_fine: int = 40, n_superfine: int = 80, device: str = "cuda"):
        super().__init__(n_coarse, n_fine, device)
        self.n_superfine = n_superfine
        self.x_superfine = np.linspace(0, 1, n_superfine)
        self.y_superfine = np.linspace(0, 1, n_superfine)
        self.X_superfine, self.Y_superfine = np.meshgrid(self.x_superfine, self.y_superfine)

    @property
    def L_superfine(self):
        return self._create_laplacian(self.n_superfine)

    def generate_forcing_term_superfine(self, k1: float, k2: float) -> np.ndarray:
        return P.forcing_batched(np.array([[k1, k2]]), self.n_superfine, self.device)[0].cpu().numpy()

    def solve_poisson_superfine(self, f: np.ndarray, theta: np.ndarray) -> np.ndarray:
        n = self.n_superfine
        return P.solve_batched(np.asarray(f, np.float64).reshape(n, n), np.asarray(theta, np.float64).reshape(n, n),
                               device=self.device)[0].cpu().numpy()

    def extract_subdomain(self, field, start_x: int, start_y: int, size: int):
        return field[start_y:start_y + size, start_x:start_x + size]

    def downsample(self, field, factor: int = 2):
        return field[::factor, ::factor]

    def generate_subdomain_dataset(self, n_samples: int, k_range: Tuple[float, float] = (0.5, 12.0),
                                   keep_on_device: bool = False, shard=None) -> dict:
        """enhanced_data_generation.py:98-165 with one batched 80^2 solve.  ``keep_on_device`` /
        ``shard``: as PoissonSolver.generate_dataset (draws stay global, solves are sharded)."""
        n_all, nf, nsf = n_samples, self.n_fine, self.n_superfine
        k_all = np.empty((n_all, 2))
        starts_all = np.empty((n_all, 2), dtype=np.int64)
        max_start = nsf - nf
        for s in range(n_all):  # reference draw order: k1, k2, start_x, start_y
            k_all[s, 0] = np.random.uniform(*k_range)
            k_all[s, 1] = np.random.uniform(*k_range)
            starts_all[s, 0] = np.random.randint(0, max_start)
            starts_all[s, 1] = np.random.randint(0, max_start)
        rank, world = resolve_shard(shard)
        lo, hi = shard_range(n_all, rank, world)
        k, starts, ns = k_all[lo:hi], starts_all[lo:hi], hi - lo
        f_sf = P.forcing_batched(k, nsf, self.device)
        th_sf = torch.ones(ns, nsf, nsf, dtype=torch.float64, device=self.device)
        u_sf = P.solve_batched(f_sf, th_sf, device=self.device)
        # crop windows by one gather: rows start_y + i, cols start_x + j
        ar = torch.arange(nf, device=self.device)
        sx = torch.as_tensor(starts[:, 0], device=self.device)
        sy = torch.as_tensor(starts[:, 1], device=self.device)
        rows = (sy[:, None] + ar[None, :])[:, :, None].expand(ns, nf, nf)
        cols = (sx[:, None] + ar[None, :])[:, None, :].expand(ns, nf, nf)
        bidx = torch.arange(ns, device=self.device)[:, None, None].expand(ns, nf, nf)
        crop = lambda a: a[bidx, rows, cols]  # noqa: E731
        f_fine, u_fine, th_fine = crop(f_sf), crop(u_sf), crop(th_sf)
        out = {
            "u_coarse": u_fine[:, ::2, ::2],
            "u_fine": u_fine,
            "f_coarse": f_fine[:, ::2, ::2],
            "f_fine": f_fine,
            "theta_coarse": th_fine[:, ::2, ::2],
            "theta_fine": th_fine,
        }
        out = {kk: v.contiguous() for kk, v in out.items()}
        host = {"k1": k_all[:, 0].copy(), "k2": k_all[:, 1].copy(), "is_subdomain": np.ones(n_all, dtype=bool)}
        out = gather_fields(out, n_all, world, tuple(host), host)
        return out if keep_on_device else to_numpy(out)

    def combine_datasets(self, dataset1: Dict, dataset2: Dict) -> Dict:
        """enhanced_data_generation.py:167-191.  Device tensors are concatenated on the device
        (torch.cat), host arrays with np.concatenate: the fields of keep_on_device datasets never
        leave HBM on their way to PDEDataset."""
        if "is_subdomain" not in dataset1:
            dataset1["is_subdomain"] = np.zeros(len(dataset1["u_fine"]), dtype=bool)
        out = {}
        for key in dataset1:
            if key not in dataset2:
                out[key] = dataset1[key]
            elif isinstance(dataset1[key], torch.Tensor) or isinstance(dataset2[key], torch.Tensor):
                a, b = dataset1[key], dataset2[key]
                dev = a.device if isinstance(a, torch.Tensor) else b.device
                out[key] = torch.cat([torch.as_tensor(a, device=dev), torch.as_tensor(b, device=dev)])
            else:
                out[key] = np.concatenate([dataset1[key], dataset2[key]])
        return out


if __name__ == "__main__":
    from pathlib import Path
    solver = EnhancedPoissonSolver(20, 40, 80)
    path = Path("data") / "pde_dataset.npz"
    if path.exists():
        existing = dict(np.load(path))
    else:
        existing = solver.generate_dataset(n_samples=1000, k_range=(0.5, 5.0))
    sub = solver.generate_subdomain_dataset(n_samples=1000, k_range=(0.5, 12.0))
    solver.save_dataset(solver.combine_datasets(existing, sub))
    print("Combined dataset saved successfully!")
