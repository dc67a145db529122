"""Batched on-device Poisson solve: the HIP replacement of scipy spsolve on the 5-point
operator (reference src/data_generation.py:35-104, src/enhanced_data_generation.py:47-68).

``solve_batched(f, theta)`` solves theta * Lap_h(u) = f for B problems of size n x n
(h = 1/(n-1), all n^2 nodes unknown, zero ghost ring -- exactly diag(theta) @ L of the
reference) as the SPD system (-L) u = -f/theta by matrix-free CG in fp64:
  * n <= 128 : one workgroup per problem, direction vector in LDS (one launch);
  * n  > 128 : grid CG, two launches per iteration; the host polls a device `done` flag
               every ``check_every`` iterations (the only host sync of the path).
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
                  return_iters: bool = False, check_every: int = 128):
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
    if n <= int(query("srpde_poisson_lds_max_n")):
        call("srpde_poisson_cg_lds", f.data_ptr(), theta.data_ptr(), u.data_ptr(), B, n, float(rtol), int(maxit),
             iters.data_ptr(), 0, stream_ptr())
    else:
        ws_bytes = int(query("srpde_poisson_workspace_size", B, n))
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=device)
        call("srpde_poisson_cg_grid_init", f.data_ptr(), theta.data_ptr(), B, n, ws.data_ptr(), ws_bytes,
             stream_ptr())
        done_off = int(query("srpde_poisson_cg_grid_done_offset", B, n))
        done = ws[done_off:done_off + 4 * B].view(torch.int32)
        k = 0
        while k < maxit + 1:
            cnt = min(check_every, maxit + 1 - k)
            call("srpde_poisson_cg_grid_iterate", B, n, float(rtol), k, cnt, int(maxit), ws.data_ptr(), ws_bytes,
                 stream_ptr())
            k += cnt
            if bool((done != 0).all()):  # host poll (one small D2H copy per chunk)
                break
        call("srpde_poisson_cg_grid_finish", u.data_ptr(), iters.data_ptr(), B, n, int(maxit), ws.data_ptr(),
             ws_bytes, stream_ptr())
    return (u, iters) if return_iters else u
