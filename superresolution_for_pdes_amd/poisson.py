"""Batched on-device Poisson solve: the HIP replacement of scipy spsolve on the 5-point
operator (reference src/data_generation.py:35-104, src/enhanced_data_generation.py:47-68).

``solve_batched(f, theta)`` solves theta * Lap_h(u) = f for B problems of size n x n
(h = 1/(n-1), all n^2 nodes unknown, zero ghost ring -- exactly diag(theta) @ L of the
reference) as the SPD system (-L) u = -f/theta by matrix-free CG in fp64:
  * n <= 128 : one workgroup per problem, direction vector in LDS (one launch);
  * n  > 128 : grid CG as cooperative launches (srpde_poisson_coop_problems(n) problems each):
               two grid barriers per iteration instead of two launches, convergence decided on
               the device -- stream-ordered, no host sync.
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
    if k.shape[0] == 0:      # an empty rank shard (shard_range with n < world): nothing to launch
        return out
    call("srpde_forcing_batched", k.data_ptr(), k.shape[0], n, out.data_ptr(), stream_ptr())
    return out


class GridBarrierAbort(RuntimeError):
    """A cooperative grid-CG launch gave up at a grid barrier (iters = -1): its u is not a solution."""


def solve_batched(f, theta, rtol: float = DEFAULT_RTOL, maxit: int = None, device="cuda",
                  return_iters: bool = False, check: bool = True, _start_aborted: bool = False):
    """u[B, n, n] (float64, on device) with theta*Lap(u) = f per problem.

    For n above the LDS solver's limit the solve runs as cooperative launches whose grid barriers
    abort after ~1 s of waiting (srpde_poisson_cg_batched marks those problems iters = -1 and
    leaves u unconverged).  ``check`` (default) reads the iteration counts back -- one host sync,
    only on that path, not under stream capture -- and raises GridBarrierAbort instead of returning
    such a u (every data-generation caller otherwise consumed it silently)."""
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
    if B == 0:               # an empty rank shard: the C entry rejects B = 0, there is nothing to solve
        return (u, iters) if return_iters else u
    ws_bytes = int(query("srpde_poisson_workspace_size", B, n))
    ws = torch.empty(max(ws_bytes, 16), dtype=torch.uint8, device=device)
    # (_start_aborted, a test hook: the C entry's negative rtol -- every grid-CG launch starts aborted)
    call("srpde_poisson_cg_batched", f.data_ptr(), theta.data_ptr(), u.data_ptr(), B, n,
         -float(rtol) if _start_aborted else float(rtol), int(maxit),
         iters.data_ptr(), ws.data_ptr(), ws_bytes, stream_ptr())
    if check and n > int(query("srpde_poisson_lds_max_n")) and not torch.cuda.is_current_stream_capturing():
        bad = int((iters < 0).sum())
        if bad:
            raise GridBarrierAbort(f"srpde_poisson_cg_batched: {bad} of {B} problems (n={n}) aborted at a grid "
                                   "barrier; their u is not a solution")
    return (u, iters) if return_iters else u


def solve_rows_sharded(f, theta, rtol: float = DEFAULT_RTOL, maxit: int = None, device="cuda", group=None,
                       check_every: int = 64, return_iters: bool = False):
    """ONE n x n problem (theta*Lap(u) = f) with its rows sharded over the ranks of ``group``
    (the ground-truth solve of solve_multi_resolution, resolution_comparison.py:62-73):
    every rank passes the whole f / theta (the seeded draws are replicated), solves the rows
    shard_range(n, rank, world) with the srpde_poisson_rows_* kernels -- per iteration two launches
    and two all-gathers (one scalar, then the rank's <r,r> partial with its first / last rows of r and
    p, which is what the neighbours' stencils need) -- and all ranks return the full u[n, n].  At
    world 1 (no process group) it runs the same kernels without collectives."""
    import torch.distributed as dist

    from .data_generation import shard_range
    dist_on = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size(group) if dist_on else 1
    rank = dist.get_rank(group) if dist_on else 0
    f = _dev_f64(f, device)
    theta = _dev_f64(theta, device)
    if theta.shape != f.shape:
        theta = theta.expand_as(f).contiguous()
    n = f.shape[-1]
    if f.dim() != 2 or f.shape[0] != n:
        raise ValueError("one square problem [n, n]")
    if world > n:
        raise ValueError(f"more ranks ({world}) than grid rows ({n})")
    if maxit is None:
        maxit = 20 * n * n
    lo, hi = shard_range(n, rank, world)
    nloc = hi - lo
    fl, tl = f[lo:hi].contiguous(), theta[lo:hi].contiguous()
    ws_bytes = int(query("srpde_poisson_rows_workspace_size", n, nloc))
    ws = torch.zeros(ws_bytes, dtype=torch.uint8, device=device)
    done_at = int(query("srpde_poisson_rows_done_offset", n, nloc))
    done = ws[done_at:done_at + 4].view(torch.int32)
    send = torch.zeros(4 * n + 1, dtype=torch.float64, device=device)
    spq = torch.zeros(1, dtype=torch.float64, device=device)
    if world > 1:
        gath = torch.zeros(world, 4 * n + 1, dtype=torch.float64, device=device)
        gpq = torch.zeros(world, 1, dtype=torch.float64, device=device)
        gath_parts, gpq_parts = list(gath.unbind(0)), list(gpq.unbind(0))

        def gather_send():
            dist.all_gather(gath_parts, send, group=group)

        def gather_pq():
            dist.all_gather(gpq_parts, spq, group=group)
    else:
        gath, gpq = send, spq
        gather_send = gather_pq = (lambda: None)
    sp = stream_ptr()
    call("srpde_poisson_rows_init", fl.data_ptr(), tl.data_ptr(), n, nloc, ws.data_ptr(), ws_bytes,
         send.data_ptr(), sp)
    gather_send()
    for k in range(maxit + 1):
        call("srpde_poisson_rows_iter_a", n, nloc, lo, rank, world, gath.data_ptr(), k, int(maxit), float(rtol),
             ws.data_ptr(), ws_bytes, spq.data_ptr(), sp)
        gather_pq()
        call("srpde_poisson_rows_iter_b", n, nloc, world, gath.data_ptr(), gpq.data_ptr(), k, ws.data_ptr(),
             ws_bytes, send.data_ptr(), sp)
        gather_send()
        # every rank decides convergence from the same gathered values, so all leave together
        if (k + 1) % check_every == 0 and int(done.item()):
            break
    ul = torch.empty(nloc, n, dtype=torch.float64, device=device)
    it = torch.zeros(1, dtype=torch.int32, device=device)
    call("srpde_poisson_rows_finish", ul.data_ptr(), it.data_ptr(), n, nloc, int(maxit), ws.data_ptr(), ws_bytes, sp)
    if world > 1:
        counts = [shard_range(n, r, world) for r in range(world)]
        cmax = max(b - a for a, b in counts)
        pad = torch.zeros(cmax, n, dtype=torch.float64, device=device)
        pad[:nloc] = ul
        parts = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(parts, pad, group=group)
        u = torch.cat([parts[r][:b - a] for r, (a, b) in enumerate(counts)])
    else:
        u = ul
    return (u, int(it.item())) if return_iters else u
