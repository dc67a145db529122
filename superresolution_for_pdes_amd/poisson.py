"""Batched on-device Poisson solve: the HIP replacement of scipy spsolve on the 5-point
operator (reference src/data_generation.py:35-104, src/enhanced_data_generation.py:47-68).

``solve_batched(f, theta)`` solves theta * Lap_h(u) = f for B problems of size n x n
(h = 1/(n-1), all n^2 nodes unknown, zero ghost ring -- exactly diag(theta) @ L of the
reference) as the SPD system (-L) u = -f/theta by matrix-free CG in fp64:
  * n <= 128 : one workgroup per problem, direction vector in LDS (one launch);
  * n  > 128 : grid CG, two launches per iteration; the host polls a device `done` flag
               every 128 iterations (the only host sync of the path).
Both go through the single C entry ``srpde_poisson_cg_batched`` (include/srpde.h), which a
non-Python caller binds the same way.
"""
from __future__ import annotations

import numpy as np
import torch

from ._lib import call, query, stream_ptr

DEFAULT_RTOL = 1e-12


def _dev_f64(a, device):
    if isinstance(a, torch.Tensor):
        return a.to(device=device, dtype=torch.float64).contiguous()
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(device)


def forcing_batched(k12, n: int, device="cuda"):
    """f[b] = sin(2 pi k1_b X) sin(2 pi k2_b Y) on linspace(0,1,n)^2 (data_generation.py:60-77)."""
    k = _dev_f64(k12, device).reshape(-1, 2).contiguous()
    out = torch.empty(k.shape[0], n, n, dtype=torch.float64, device=device)
    call("srpde_forcing_batched", k.data_ptr(), k.shape[0], n, out.data_ptr(), stream_ptr())
    return out


def solve_batched(f, theta, rtol: float = DEFAULT_RTOL, maxit: int = None, device="cuda",
                  return_iters: bool = False):
    """u[B, n, n] (float64, on device) with theta*Lap(u) = f per problem."""
    f = _dev_f64(f, device)
    theta = _dev_f64(theta, device)
    if f.dim() == 2:
        f, theta = f.unsqueeze(0), theta.unsqueeze(0)
    if theta.shape != f.shape:
        theta = theta.expand_as(f).contiguous()
    B, n, n2 = f.shape
    if n != n2:
        raise ValueError("square grids only")
    if maxit is None:
        maxit = 20 * n * n
    u = torch.empty_like(f)
    iters = torch.empty(B, dtype=torch.int32, device=device)
    ws_bytes = int(query("srpde_poisson_workspace_size", B, n))
    ws = torch.empty(max(ws_bytes, 16), dtype=torch.uint8, device=device)
    call("srpde_poisson_cg_batched", f.data_ptr(), theta.data_ptr(), u.data_ptr(), B, n, float(rtol), int(maxit),
         iters.data_ptr(), ws.data_ptr(), ws_bytes, stream_ptr())
    return (u, iters) if return_iters else u
