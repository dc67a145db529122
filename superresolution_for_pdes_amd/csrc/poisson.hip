// Batched matrix-free conjugate-gradient Poisson solver (fp64) for gfx950.
//
// Reference: PoissonSolver._create_laplacian + solve_poisson (src/data_generation.py:35-58,
// :79-104) assemble diag(theta) @ L (5-point, all n^2 nodes are unknowns, zero ghost ring
// outside the grid, h = 1/(n-1)) and call scipy spsolve (SuperLU).  theta only scales rows,
// so the system is equivalent to the SPD problem
//           (-L) u = -f / theta
// which is solved here by CG on a matrix-free stencil, for B independent problems at once.
//
// * n <= 128  : one workgroup per problem, Chronopoulos-Gear CG: the residual r (with its zero
//               ghost ring) lives in LDS, x / r / p / s / w stay in registers (NPT points per
//               lane); 2 barriers per iteration (one fused two-value reduction on the DPP network),
//               deterministic fixed-order block reductions.
// * n  > 128  : grid CG, 2 launches per iteration (A: beta, p <- r + beta p, q = A p, <p,q>
//               partials;  B: alpha, x += alpha p, r -= alpha A p, <r,r> partials); every
//               block re-reduces the previous launch's partials in the same order, so all
//               blocks agree on alpha/beta without a grid barrier or host round trip.
//               A sticky per-problem `done` flag makes extra launches no-ops.
#include <map>
#include <mutex>
#include <tuple>
#include <atomic>
#include "common.h"

#include <vector>

namespace srpde {

constexpr int CG_MAXT = 1024;

// fp64 wave reduction on the DPP network (no LDS round trips): butterfly within quads, rotations
// within 16-lane rows, then the GFX9 row broadcasts fold the four rows into lane 63, read back as a
// wave-uniform value.  Fixed order: every wave of every block sums identically.
// FULL: the pattern writes every lane, so no `old` operand is needed (mov_dpp: no zeroing or copy
// move before it); the row broadcasts write only the masked rows and keep 0 elsewhere
template <int CTRL, int ROWS, bool FULL = true>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  if (FULL)
    return __hiloint2double(__builtin_amdgcn_mov_dpp(hi, CTRL, ROWS, 0xf, false),
                            __builtin_amdgcn_mov_dpp(lo, CTRL, ROWS, 0xf, false));
  return __hiloint2double(__builtin_amdgcn_update_dpp(0, hi, CTRL, ROWS, 0xf, false),
                          __builtin_amdgcn_update_dpp(0, lo, CTRL, ROWS, 0xf, false));
}
// the sum of lanes 0..15 (the rest contribute 0), wave-uniform
__device__ __forceinline__ double row0_sum_dpp(double v) {
  v += dpp_f64<0xB1, 0xf>(v);
  v += dpp_f64<0x4E, 0xf>(v);
  v += dpp_f64<0x124, 0xf>(v);
  v += dpp_f64<0x128, 0xf>(v);
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), 0), hi = __builtin_amdgcn_readlane(__double2hiint(v), 0);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double wave_sum_dpp(double v) {
  v += dpp_f64<0xB1, 0xf>(v);    // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E, 0xf>(v);    // quad_perm [2,3,0,1]
  v += dpp_f64<0x124, 0xf>(v);   // row_ror:4
  v += dpp_f64<0x128, 0xf>(v);   // row_ror:8   (every lane: its row's sum)
  v += dpp_f64<0x142, 0xa, false>(v);   // row_bcast:15 into rows 1, 3
  v += dpp_f64<0x143, 0xc, false>(v);   // row_bcast:31 into rows 2, 3 (lane 63: the wave's sum)
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), 63), hi = __builtin_amdgcn_readlane(__double2hiint(v), 63);
  return __hiloint2double(hi, lo);
}

// (a, b) summed over the block, the same values in every thread: per-wave DPP sums into `slots`
// ([2][16] doubles), one barrier, then each wave re-reduces the nw wave sums in lane order.
__device__ __forceinline__ void block_sum2(double& a, double& b, double* slots) {
  a = wave_sum_dpp(a);
  b = wave_sum_dpp(b);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = (blockDim.x + 63) >> 6;
  if (lane == 0) { slots[w] = a; slots[16 + w] = b; }
  __syncthreads();
  // nw <= 16 wave sums: one 16-lane row reduces them (same order in every wave)
  a = row0_sum_dpp(lane < nw ? slots[lane] : 0.0);
  b = row0_sum_dpp(lane < nw ? slots[16 + lane] : 0.0);
}

// The Chronopoulos-Gear scalars of the next iteration from gamma_new = <r, r>, delta_new = <A r, r>:
// beta = gamma_new / gamma, alpha = gamma_new / (delta_new - beta gamma_new / alpha) = gn c / D with
// c = gamma alpha, D = delta_new c - gamma_new^2; both from ONE division, 1 / (gamma D) (the three
// chained divisions were ~35 of an iteration's ~200 VALU instructions per wave, all on its critical
// path).  Magnitudes: gamma D ~ gamma^3, far inside fp64's range for rtol >= 1e-30.
__device__ __forceinline__ void cg_scalars(double gn, double dn, double& gamma, double& alpha, double& beta) {
  const double c = gamma * alpha;
  const double D = dn * c - gn * gn;
  const double rr = 1.0 / (gamma * D);
  beta = gn * D * rr;
  alpha = gn * c * gamma * rr;
  gamma = gn;
}

// Chronopoulos-Gear CG (the same Krylov iterates as textbook CG, rearranged so that both inner
// products of an iteration, gamma = <r, r> and delta = <A r, r>, come from ONE block reduction):
//   w = A r;  gamma, delta;  beta = gamma / gamma_old;  alpha = gamma / (delta - beta * gamma / alpha_old)
//   p = r + beta p;  s = w + beta s  (= A p);  x += alpha p;  r -= alpha s
// Two barriers per iteration (r visible for the stencil; the reduction) against textbook CG's three;
// r lives in LDS with its zero ghost ring, x / r / p / s / w in registers (NPT points per lane).
template <int NPT>
__global__ __launch_bounds__(CG_MAXT) void cg_lds_kernel(const double* __restrict__ f,
                                                         const double* __restrict__ theta, double* __restrict__ u,
                                                         int n, double rtol, int maxit, int* __restrict__ iters,
                                                         double* __restrict__ resid) {
  extern __shared__ double sp[];
  const int N2 = n * n, ld = n + 2;
  double* rl = sp;                       // (n+2)^2
  double* slots = sp + ld * ld;          // [2][2][16]: reduction parity x (gamma, delta) x wave
  const size_t off = (size_t)blockIdx.x * N2;
  const double inv_h2 = (double)(n - 1) * (double)(n - 1);
  const int T = blockDim.x;

  for (int e = threadIdx.x; e < ld * ld; e += T) rl[e] = 0.0;
  double x[NPT], r[NPT], p[NPT], s[NPT], w[NPT];
  int li[NPT];
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int i = threadIdx.x + k * T;
    x[k] = 0.0; p[k] = 0.0; s[k] = 0.0; w[k] = 0.0;
    if (i < N2) {
      const int yy = i / n, xx = i - yy * n;
      li[k] = yy * ld + xx;   // the point's up-left corner in rl: every neighbour at a positive offset
      r[k] = -f[off + i] / theta[off + i];
    } else {
      li[k] = -1;
      r[k] = 0.0;
    }
  }
  __syncthreads();  // ghost ring zeroed before interior writes
  int par = 0;
  // w = A r and (gamma, delta) of the current r (r already written to rl, one barrier passed)
  auto apply_reduce = [&](double& gamma, double& delta) {
    double g = 0.0, d = 0.0;
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      if (li[k] >= 0) {
        const double* q = rl + li[k];
        w[k] = (4.0 * r[k] - q[ld] - q[ld + 2] - q[1] - q[2 * ld + 1]) * inv_h2;
        g += r[k] * r[k];
        d += w[k] * r[k];
      }
      // two points' neighbour loads in flight at a time: hoisting all of them spills the five
      // register vectors (the block's other waves hide the LDS latency)
      if (k & 1) __builtin_amdgcn_sched_barrier(0);
    }
    block_sum2(g, d, slots + 32 * par);
    par ^= 1;
    gamma = g;
    delta = d;
  };
#pragma unroll
  for (int k = 0; k < NPT; ++k)
    if (li[k] >= 0) rl[li[k] + ld + 1] = r[k];
  __syncthreads();
  double gamma, delta;
  apply_reduce(gamma, delta);
  const double stop = rtol * rtol * gamma;
  const double g0 = gamma;
  double alpha = gamma / delta, beta = 0.0;
  int it = 0;
  auto step = [&]() {
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      p[k] = r[k] + beta * p[k];
      s[k] = w[k] + beta * s[k];
      x[k] += alpha * p[k];
      r[k] -= alpha * s[k];
      if (li[k] >= 0) rl[li[k] + ld + 1] = r[k];
    }
    ++it;
    __syncthreads();   // r visible to the neighbours' stencils (all reads of the old r are done:
                       // they precede the reduction barrier every thread has passed)
    double gn, dn;
    apply_reduce(gn, dn);
    cg_scalars(gn, dn, gamma, alpha, beta);
  };
  // two iterations per trip: one per trip rotated the loop-carried vectors through register copies
  while (gamma > stop && it < maxit) {
    step();
    if (!(gamma > stop && it < maxit)) break;
    step();
  }
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int i = threadIdx.x + k * T;
    if (i < N2) u[off + i] = x[k];
  }
  if (threadIdx.x == 0) {
    if (iters) iters[blockIdx.x] = it;
    if (resid) resid[blockIdx.x] = sqrt(gamma / (g0 > 0.0 ? g0 : 1.0));
  }
}

// cg_lds_kernel with the grid size a compile-time constant (used at n = 80):
// T = (T / n) rows of n points per slab, point k of a lane NPT = ceil(n / (T / n)) slabs down, so one
// LDS address register serves all of a lane's points and every neighbour read is an immediate offset
// (the generic kernel held NPT addresses and spilled at n = 80: 19 VGPRs, scratch reloads inside the
// stencil).  Same recurrence, expressions and reduction order as cg_lds_kernel.
template <int N, int T>
__global__ __launch_bounds__(T) void cg_lds_n_kernel(const double* __restrict__ f, const double* __restrict__ theta,
                                                     double* __restrict__ u, double rtol, int maxit,
                                                     int* __restrict__ iters, double* __restrict__ resid) {
  constexpr int LD = N + 2, RPS = T / N, NPT = (N + RPS - 1) / RPS, SLAB = RPS * LD, N2 = N * N;
  static_assert(T % N == 0 && T % 64 == 0 && T <= CG_MAXT, "slab layout");
  __shared__ double rl[LD * LD];
  __shared__ double slots[64];
  const size_t off = (size_t)blockIdx.x * N2;
  const double inv_h2 = (double)(N - 1) * (double)(N - 1);
  const int tid = threadIdx.x, row = tid / N, col = tid - row * N;
  const bool last_ok = (NPT - 1) * RPS + row < N;   // points k < NPT - 1 always exist
  double* qb = rl + row * LD + col;                 // point k's up-left corner: qb + k * SLAB

  for (int e = tid; e < LD * LD; e += T) rl[e] = 0.0;
  double x[NPT], r[NPT], p[NPT], s[NPT], w[NPT];
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    x[k] = 0.0; p[k] = 0.0; s[k] = 0.0; w[k] = 0.0;
    r[k] = (k < NPT - 1 || last_ok) ? -f[off + tid + k * T] / theta[off + tid + k * T] : 0.0;
  }
  __syncthreads();   // ghost ring zeroed before interior writes
  int par = 0;
  auto apply_reduce = [&](double& gamma, double& delta) {
    double g = 0.0, d = 0.0;
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      if (k < NPT - 1 || last_ok) {
        const double* q = qb + k * SLAB;
        w[k] = (4.0 * r[k] - q[LD] - q[LD + 2] - q[1] - q[2 * LD + 1]) * inv_h2;
        g += r[k] * r[k];
        d += w[k] * r[k];
      }
    }
    block_sum2(g, d, slots + 32 * par);
    par ^= 1;
    gamma = g;
    delta = d;
  };
#pragma unroll
  for (int k = 0; k < NPT; ++k)
    if (k < NPT - 1 || last_ok) qb[k * SLAB + LD + 1] = r[k];
  __syncthreads();
  double gamma, delta;
  apply_reduce(gamma, delta);
  const double stop = rtol * rtol * gamma;
  const double g0 = gamma;
  double alpha = gamma / delta, beta = 0.0;
  int it = 0;
  auto step = [&]() {
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      p[k] = r[k] + beta * p[k];
      s[k] = w[k] + beta * s[k];
      x[k] += alpha * p[k];
      r[k] -= alpha * s[k];
      if (k < NPT - 1 || last_ok) qb[k * SLAB + LD + 1] = r[k];
    }
    ++it;
    __syncthreads();
    double gn, dn;
    apply_reduce(gn, dn);
    cg_scalars(gn, dn, gamma, alpha, beta);
  };
  // two iterations per trip: the loop-carried vectors keep their registers (one iteration per trip
  // rotated them through copies, ~45 moves per iteration)
  while (gamma > stop && it < maxit) {
    step();
    if (!(gamma > stop && it < maxit)) break;
    step();
  }
#pragma unroll
  for (int k = 0; k < NPT; ++k)
    if (k < NPT - 1 || last_ok) u[off + tid + k * T] = x[k];
  if (tid == 0) {
    if (iters) iters[blockIdx.x] = it;
    if (resid) resid[blockIdx.x] = sqrt(gamma / (g0 > 0.0 ? g0 : 1.0));
  }
}

// ------------------------------- grid CG (n > 128) --------------------------------
struct GridCG {
  double *x, *r, *p0, *p1;  // [B][N2]
  double *rrp0, *rrp1, *pqp, *bbp;  // [B][nb]
  int* done;    // [B]
  int* iters;   // [B]
  int n, nb, B;
  double rtol;
};

// 512 threads x 4 points: 2048 points per block (a 640^2 problem is 200 blocks; 143 VGPRs, no spill)
constexpr int GCG_T = 512, GCG_NPT = 4, GCG_PTS = GCG_T * GCG_NPT;

__device__ __forceinline__ double sum_parts(const double* part, int nb, double* sh) {
  double s = 0.0;
  for (int k = threadIdx.x; k < nb; k += blockDim.x) s += part[k];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  double t = 0.0;
  for (int k = 0; k < (int)(blockDim.x >> 6); ++k) t += sh[k];
  __syncthreads();
  return t;
}

__device__ __forceinline__ void write_part(double v, double* sh, double* dst) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) t += sh[k];
    *dst = t;
  }
}

__global__ __launch_bounds__(GCG_T) void gcg_init_kernel(const double* __restrict__ f,
                                                         const double* __restrict__ theta, GridCG g) {
  __shared__ double sh[8];
  const int b = blockIdx.y, N2 = g.n * g.n;
  const size_t off = (size_t)b * N2;
  double s = 0.0;
  for (int k = 0; k < GCG_NPT; ++k) {
    const int i = blockIdx.x * GCG_PTS + k * GCG_T + threadIdx.x;
    if (i < N2) {
      const double rv = -f[off + i] / theta[off + i];
      g.x[off + i] = 0.0; g.r[off + i] = rv; g.p0[off + i] = 0.0; g.p1[off + i] = 0.0;
      s += rv * rv;
    }
  }
  write_part(s, sh, g.rrp0 + (size_t)b * g.nb + blockIdx.x);
  if (threadIdx.x == 0) g.bbp[(size_t)b * g.nb + blockIdx.x] = 0.0;  // filled by copy below
  if (blockIdx.x == 0 && threadIdx.x == 0) { g.done[b] = 0; g.iters[b] = 0; }
}

__global__ void gcg_copy_bb_kernel(GridCG g) {
  const int b = blockIdx.y;
  for (int k = threadIdx.x; k < g.nb; k += blockDim.x) g.bbp[(size_t)b * g.nb + k] = g.rrp0[(size_t)b * g.nb + k];
}

// launch A of iteration k
__global__ __launch_bounds__(GCG_T) void gcg_a_kernel(GridCG g, int k, int maxit) {
  __shared__ double sh[8];
  const int b = blockIdx.y, n = g.n, N2 = n * n;
  if (g.done[b]) return;
  const double* rr_cur = (k & 1) ? g.rrp1 : g.rrp0;
  const double* rr_old = (k & 1) ? g.rrp0 : g.rrp1;
  const double rr = sum_parts(rr_cur + (size_t)b * g.nb, g.nb, sh);
  const double bb = sum_parts(g.bbp + (size_t)b * g.nb, g.nb, sh);
  if (rr <= g.rtol * g.rtol * bb || k >= maxit) {
    if (blockIdx.x == 0 && threadIdx.x == 0) { g.done[b] = 1; g.iters[b] = k; }
    return;
  }
  const double beta = k == 0 ? 0.0 : rr / sum_parts(rr_old + (size_t)b * g.nb, g.nb, sh);
  const size_t off = (size_t)b * N2;
  const double* po = ((k & 1) ? g.p1 : g.p0) + off;
  double* pn = ((k & 1) ? g.p0 : g.p1) + off;
  const double* rv = g.r + off;
  const double inv_h2 = (double)(n - 1) * (double)(n - 1);
  double s = 0.0;
  for (int kk = 0; kk < GCG_NPT; ++kk) {
    const int i = blockIdx.x * GCG_PTS + kk * GCG_T + threadIdx.x;
    if (i < N2) {
      const int yy = i / n, xx = i - yy * n;
      auto pv = [&](int j) { return rv[j] + beta * po[j]; };
      const double pc = pv(i);
      double nb = 0.0;
      if (xx > 0) nb += pv(i - 1);
      if (xx < n - 1) nb += pv(i + 1);
      if (yy > 0) nb += pv(i - n);
      if (yy < n - 1) nb += pv(i + n);
      const double qv = (4.0 * pc - nb) * inv_h2;
      pn[i] = pc;
      s += pc * qv;
    }
  }
  write_part(s, sh, g.pqp + (size_t)b * g.nb + blockIdx.x);
}

// launch B of iteration k
__global__ __launch_bounds__(GCG_T) void gcg_b_kernel(GridCG g, int k) {
  __shared__ double sh[8];
  const int b = blockIdx.y, n = g.n, N2 = n * n;
  if (g.done[b]) return;
  const double* rr_cur = (k & 1) ? g.rrp1 : g.rrp0;
  double* rr_next = (k & 1) ? g.rrp0 : g.rrp1;
  const double rr = sum_parts(rr_cur + (size_t)b * g.nb, g.nb, sh);
  const double pq = sum_parts(g.pqp + (size_t)b * g.nb, g.nb, sh);
  const double alpha = rr / pq;
  const size_t off = (size_t)b * N2;
  const double* pn = ((k & 1) ? g.p0 : g.p1) + off;
  double* xv = g.x + off;
  double* rv = g.r + off;
  const double inv_h2 = (double)(n - 1) * (double)(n - 1);
  double s = 0.0;
  for (int kk = 0; kk < GCG_NPT; ++kk) {
    const int i = blockIdx.x * GCG_PTS + kk * GCG_T + threadIdx.x;
    if (i < N2) {
      const int yy = i / n, xx = i - yy * n;
      double nb = 0.0;
      if (xx > 0) nb += pn[i - 1];
      if (xx < n - 1) nb += pn[i + 1];
      if (yy > 0) nb += pn[i - n];
      if (yy < n - 1) nb += pn[i + n];
      const double pc = pn[i];
      const double qv = (4.0 * pc - nb) * inv_h2;
      xv[i] += alpha * pc;
      const double rn = rv[i] - alpha * qv;
      rv[i] = rn;
      s += rn * rn;
    }
  }
  write_part(s, sh, rr_next + (size_t)b * g.nb + blockIdx.x);
}

__global__ void gcg_finish_kernel(GridCG g, double* __restrict__ u, int* __restrict__ iters, int maxit) {
  const int b = blockIdx.y, N2 = g.n * g.n;
  const size_t off = (size_t)b * N2;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < N2; i += gridDim.x * blockDim.x) u[off + i] = g.x[off + i];
  if (blockIdx.x == 0 && threadIdx.x == 0 && iters) iters[b] = g.done[b] ? g.iters[b] : maxit;
}

// ---------------- grid CG in ONE cooperative launch (n > 128, stream-ordered) ----------------
// The same iteration as gcg_a / gcg_b (same per-block partial sums, same re-reduction order, same
// expressions: bit-identical iterates) with the two launch boundaries of an iteration replaced by
// two grid barriers, so the solve is one launch and the host never polls.  Every block owns GCG_PTS
// consecutive points of one problem; x, r, p and q of its points stay in registers, the new p also in
// LDS for the in-block stencil, and only the first / last n points' r and p (p double-buffered by
// parity) go to global memory for the neighbouring blocks.  All blocks co-reside
// (hipLaunchCooperativeKernel checks it); a problem that converges keeps its blocks at the barriers
// until every problem of the launch has (ctl[0] counts them), and every block leaves the loop at the
// same barrier.  A barrier that waits longer than ~1 s sets ctl[1] (abort), which releases every
// waiter: the launch then ends with iters = -1 instead of hanging the queue.
// The grid barrier is a two-level tree of monotonic arrival counters (zeroed before the launch):
// bar[1 + g] counts the arrivals of block group g (COOP_GRP consecutive blocks), the last arriver of
// a group bumps bar[0], and every block waits for bar[0] to reach epoch x groups -- COOP_GRP + groups
// serialised atomics per barrier instead of one per block on a single address.
#ifndef SRPDE_COOP_GRP
#define SRPDE_COOP_GRP 4
#endif
constexpr int COOP_GRP = SRPDE_COOP_GRP;   // A/B builds override it
struct GridCoop {
  double *er[2], *ew[2], *es[2];   // [B][N2] by parity: r, w = A r, s = A p at a block's edge points
  double *gp[2], *dp[2];           // [B][nb] by parity: per-block partials of gamma = <r, r>, delta = <w, r>
  unsigned long long* bar;      // [0] groups arrived, [1 + g] blocks of group g arrived
  unsigned* ctl;                // [0] problems converged, [1] abort
  int n, nb, B, ngrp;
  double rtol;
};

// Everything one block writes and another reads (r, p, the partials) goes through agent-scope
// relaxed atomic stores / loads, which bypass the XCD-private L2 (the sc1 bit) -- so a barrier needs
// no cache maintenance: each thread drains its stores (vmcnt) before the block arrives, and the loads
// after the barrier fetch from the coherent level.  (An agent-scope fence per block and barrier
// instead writes back and invalidates the whole L2 of its XCD: measured 14x slower at n = 640.)
__device__ __forceinline__ void st_ag(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_ag(const double* p) {
  return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ double sum_parts_ag(const double* part, int nb, double* sh) {
  double s = 0.0;
  for (int k = threadIdx.x; k < nb; k += blockDim.x) s += ld_ag(part + k);
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  double t = 0.0;
  for (int k = 0; k < (int)(blockDim.x >> 6); ++k) t += sh[k];
  __syncthreads();
  return t;
}

__device__ __forceinline__ void write_part_ag(double v, double* sh, double* dst) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) t += sh[k];
    st_ag(dst, t);
  }
}

// epoch `epoch` (1, 2, ...) of the grid barrier; false on abort (a wait past ~1 s, or the abort word
// set before the launch by srpde_poisson_cg_batched's test hook, a negative rtol).
// Memory-model assumption: the barrier pairs `s_waitcnt vmcnt(0)` after each thread's
// sc1 (L2-bypassing, agent-scope relaxed) stores with sc1 loads after the barrier, instead of an
// agent-scope release / acquire.  That is correct on gfx950 because every byte handed between blocks
// is written and read ONLY through those agent-scope atomics (st_ag / ld_ag), which are served by the
// coherent memory side and never by a CU's L1 or an XCD's L2 (MI355X_MICROARCH.md, "Valid forms":
// sc1 stores drained by vmcnt + sc1 loads behind a counter poll); it is not a guarantee of the HIP
// memory model, and a port to another target must restore the release / acquire fences.
// the poll interval of a waiting block (s_sleep units of 64 cycles); A/B builds override it
#ifndef SRPDE_COOP_SLEEP
#define SRPDE_COOP_SLEEP 2
#endif
__device__ __forceinline__ bool coop_sync(const GridCoop& g, unsigned long long epoch, int* sflag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this thread's sc1 stores have landed
  __syncthreads();
  if (threadIdx.x == 0) {
    const int grp = blockIdx.x / COOP_GRP;
    const unsigned long long gsz = min(COOP_GRP, (int)gridDim.x - grp * COOP_GRP);
    const unsigned long long old = __hip_atomic_fetch_add(g.bar + 1 + grp, 1ull, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1 == epoch * gsz) __hip_atomic_fetch_add(g.bar, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long target = epoch * (unsigned long long)g.ngrp;
    int ab = 0;
    for (unsigned spins = 0;; ++spins) {
      // the abort word first: once any block has given up, nobody passes another barrier
      if (__hip_atomic_load(g.ctl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) { ab = 1; break; }
      if (__hip_atomic_load(g.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) break;
      if (spins > (1u << 24)) {
        __hip_atomic_store(g.ctl + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ab = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(SRPDE_COOP_SLEEP);
    }
    *sflag = ab;
  }
  __syncthreads();
  asm volatile("" ::: "memory");   // no load of the next phase is hoisted above the barrier
  return *sflag == 0;
}

// Chronopoulos-Gear CG (cg_lds_kernel's recurrence) with ONE grid barrier per iteration.  After the
// barrier every block sums the (gamma, delta) partials, forms alpha / beta, updates its points
// (p = r + beta p, s = w + beta s, x += alpha p, r -= alpha s) and computes w = A r with the new r.  A
// neighbour point in another block is not read after it was updated -- that would cost a barrier --
// but recomputed from its owner's (r, w, s) of the previous iteration, stored at the owner's edge
// points, with the owner's fused expressions (so the same bits as the owner holds).  Edge values and
// partials alternate between two buffers by iteration parity: a block that is already writing
// iteration k + 1's never overwrites what a slower block still reads of iteration k.
//
// A block is 1024 threads x NPT points: p, s, w in registers, x in LDS (read once at the end), r in
// LDS with a halo of n points either side (the previous block's last row, the next block's
// first), so the stencil reads LDS only, branch-free behind a per-thread neighbour mask.  NPT = 8
// (8192-point blocks) puts 4 problems at 640^2 or 64 at 160^2 into one co-resident grid of one block
// per CU; the halo loads of an iteration are issued before its partial sums, so the two round trips
// overlap.
constexpr int GCC_T = 1024, GCC_HQ = 2;   // halo points per thread: 2 n <= 2 * 1024 (3 spilled at NPT = 8)
__host__ __device__ constexpr size_t gcc_lds_bytes(int npt, int n) {
  return ((size_t)2 * GCC_T * npt + 2 * (size_t)n) * sizeof(double);
}

template <int NPT>
__global__ __launch_bounds__(GCC_T) void gcg_coop_kernel(const double* __restrict__ f,
                                                         const double* __restrict__ theta, double* __restrict__ u,
                                                         int* __restrict__ iters, GridCoop g, int maxit) {
  constexpr int PTS = GCC_T * NPT, NW = GCC_T / 64;
  extern __shared__ double lds_d[];
  __shared__ double sh[2 * NW + 2];
  __shared__ int sflag;
  const int tid = threadIdx.x;
  const int b = blockIdx.x / g.nb, j = blockIdx.x - b * g.nb;
  const int n = g.n, N2 = n * n;
  const size_t off = (size_t)b * N2;
  const int lo = j * PTS, hi = min(N2, lo + PTS), cnt = hi - lo;
  double* rl = lds_d;               // rl[q + n]: r at point lo + q, q in [-n, cnt + n)
  double* xl = lds_d + PTS + 2 * n; // xl[q]
  unsigned long long epoch = 0;
  const double inv_h2 = (double)(n - 1) * (double)(n - 1);

  // neighbour mask, bits 4 k + (left, right, up, down) of point k
  unsigned nbm = 0;
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int q = k * GCC_T + tid;
    if (q < cnt) {
      const int i = lo + q, yy = i / n, xx = i - yy * n;
      nbm |= ((xx > 0 ? 1u : 0u) | (xx < n - 1 ? 2u : 0u) | (yy > 0 ? 4u : 0u) | (yy < n - 1 ? 8u : 0u)) << (4 * k);
    }
  }
  // halo point h of this thread: rl index and grid point (-1: outside the grid)
  int hidx[GCC_HQ], hpt[GCC_HQ];
#pragma unroll
  for (int q = 0; q < GCC_HQ; ++q) {
    const int h = tid + q * GCC_T;
    hidx[q] = h < n ? h : cnt + h;
    const int pt = h < n ? lo - n + h : hi + (h - n);
    hpt[q] = (h < 2 * n && pt >= 0 && pt < N2) ? pt : -1;
    if (h < 2 * n) rl[hidx[q]] = 0.0;
  }
  auto is_edge = [&](int q) { return q < n || q >= cnt - n; };

  // r lives in rl only (the register copy made NPT = 8 spill)
  double p[NPT], s[NPT], w[NPT];
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int q = k * GCC_T + tid;
    p[k] = 0.0; s[k] = 0.0; w[k] = 0.0;
    if (q < cnt) {
      const double r0 = -f[off + lo + q] / theta[off + lo + q];
      rl[q + n] = r0;
      xl[q] = 0.0;
      if (is_edge(q)) st_ag(g.er[0] + off + lo + q, r0);
    }
  }
  bool ok = coop_sync(g, ++epoch, &sflag);

  // w = A r from rl; (gamma, delta) partials and the edge (r, w, s) of parity `par`
  auto apply = [&](int par, int lt) {
    double gs = 0.0, ds = 0.0;
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int q = k * GCC_T + lt, c = q + n;
      if (q < cnt) {
        const unsigned m = nbm >> (4 * k);
        const double rc = rl[c];
        double acc = 0.0;
        acc += (m & 1u) ? rl[c - 1] : 0.0;
        acc += (m & 2u) ? rl[c + 1] : 0.0;
        acc += (m & 4u) ? rl[c - n] : 0.0;
        acc += (m & 8u) ? rl[c + n] : 0.0;
        w[k] = (4.0 * rc - acc) * inv_h2;
        gs += rc * rc;
        ds += w[k] * rc;
        if (is_edge(q)) {
          const size_t e = off + lo + q;
          st_ag(g.er[par] + e, rc);
          st_ag(g.ew[par] + e, w[k]);
          st_ag(g.es[par] + e, s[k]);
        }
      }
    }
    gs = wave_sum(gs);
    ds = wave_sum(ds);
    if ((tid & 63) == 0) { sh[tid >> 6] = gs; sh[NW + (tid >> 6)] = ds; }
    __syncthreads();
    if (tid == 0) {
      double tg = 0.0, td = 0.0;
#pragma unroll 1
      for (int k = 0; k < NW; ++k) { tg += sh[k]; td += sh[NW + k]; }
      st_ag(g.gp[par] + (size_t)b * g.nb + j, tg);
      st_ag(g.dp[par] + (size_t)b * g.nb + j, td);
    }
  };

  if (ok) {
#pragma unroll
    for (int q = 0; q < GCC_HQ; ++q)
      if (hpt[q] >= 0) rl[hidx[q]] = ld_ag(g.er[0] + off + hpt[q]);
    __syncthreads();
    apply(0, tid);
  }
  ok = ok && coop_sync(g, ++epoch, &sflag);
  double gamma = 0.0, stop = 0.0, alpha = 0.0, beta = 0.0;
  bool done = false;
  int it_done = maxit;
  for (int k = 0; ok; ++k) {
    const int par = k & 1;
    // per-thread offsets re-derived every iteration: hoisted, they were 64-bit addresses per array and
    // parity (NPT = 8 spilled)
    int lt = tid;
    asm volatile("" : "+v"(lt));
    int hp[GCC_HQ];
#pragma unroll
    for (int q = 0; q < GCC_HQ; ++q) { hp[q] = hpt[q]; asm volatile("" : "+v"(hp[q])); }
    double hr[GCC_HQ], hw[GCC_HQ], hs[GCC_HQ];
    if (!done) {
#pragma unroll
      for (int q = 0; q < GCC_HQ; ++q) {
        hr[q] = hw[q] = hs[q] = 0.0;
        if (hp[q] >= 0) {
          const size_t e = off + hp[q];
          hr[q] = ld_ag(g.er[par] + e);
          hw[q] = ld_ag(g.ew[par] + e);
          hs[q] = ld_ag(g.es[par] + e);
        }
      }
    }
    // both partial sums in one pass (one round trip)
    double gs = 0.0, ds = 0.0;
    for (int t = tid; t < g.nb; t += GCC_T) {
      gs += ld_ag(g.gp[par] + (size_t)b * g.nb + t);
      ds += ld_ag(g.dp[par] + (size_t)b * g.nb + t);
    }
    gs = wave_sum(gs);
    ds = wave_sum(ds);
    if ((tid & 63) == 0) { sh[tid >> 6] = gs; sh[NW + (tid >> 6)] = ds; }
    __syncthreads();
    // one thread adds the wave sums (every thread doing it held all 32 in registers: NPT = 8 spilled)
    if (tid == 0) {
      double tg = 0.0, td = 0.0;
#pragma unroll 1
      for (int t = 0; t < NW; ++t) { tg += sh[t]; td += sh[NW + t]; }
      sh[2 * NW] = tg;
      sh[2 * NW + 1] = td;
    }
    __syncthreads();
    const double gn = sh[2 * NW], dn = sh[2 * NW + 1];
    if (k == 0) {
      stop = g.rtol * g.rtol * gn;
      alpha = gn / dn;
      beta = 0.0;
    } else if (!done) {
      cg_scalars(gn, dn, gamma, alpha, beta);   // the LDS kernels' one-division form (same rounding)
    }
    if (!done) gamma = gn;
    if (!done && (gamma <= stop || k >= maxit)) {
      done = true;
      it_done = k;
      if (j == 0 && tid == 0) __hip_atomic_fetch_add(g.ctl, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!done) {
#pragma unroll
      for (int kk = 0; kk < NPT; ++kk) {
        const int q = kk * GCC_T + tid;
        if (q < cnt) {
          const double rk = rl[q + n];
          p[kk] = __builtin_fma(beta, p[kk], rk);
          s[kk] = __builtin_fma(beta, s[kk], w[kk]);
          xl[q] = __builtin_fma(alpha, p[kk], xl[q]);
          rl[q + n] = __builtin_fma(-alpha, s[kk], rk);
        }
      }
#pragma unroll
      for (int q = 0; q < GCC_HQ; ++q)
        if (hp[q] >= 0) rl[hidx[q]] = __builtin_fma(-alpha, __builtin_fma(beta, hs[q], hw[q]), hr[q]);
      __syncthreads();
      apply(par ^ 1, lt);
    }
    ok = coop_sync(g, ++epoch, &sflag);
    // every increment of ctl[0] precedes this barrier and the next one follows these reads: all
    // blocks read the same count and leave together
    if (!ok || __hip_atomic_load(g.ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (unsigned)g.B) break;
  }
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int q = k * GCC_T + tid;
    if (q < cnt) u[off + lo + q] = xl[q];
  }
  if (j == 0 && tid == 0 && iters) iters[b] = ok ? it_done : -1;
}

static GridCG carve(void* ws, int B, int n) {
  GridCG g;
  const size_t N2 = (size_t)n * n;
  g.n = n; g.B = B; g.nb = (int)((N2 + GCG_PTS - 1) / GCG_PTS);
  double* d = static_cast<double*>(ws);
  g.x = d; d += B * N2;
  g.r = d; d += B * N2;
  g.p0 = d; d += B * N2;
  g.p1 = d; d += B * N2;
  g.rrp0 = d; d += (size_t)B * g.nb;
  g.rrp1 = d; d += (size_t)B * g.nb;
  g.pqp = d; d += (size_t)B * g.nb;
  g.bbp = d; d += (size_t)B * g.nb;
  g.done = reinterpret_cast<int*>(d);
  g.iters = g.done + B;
  g.rtol = 0.0;
  return g;
}

static size_t coop_ctl_bytes(int B, int n) {   // the cooperative launches' barrier counters + ctl words
  const size_t nb = ((size_t)n * n + GCG_PTS - 1) / GCG_PTS;
  return ((B * nb + COOP_GRP - 1) / COOP_GRP + 2) * sizeof(unsigned long long);
}
static size_t grid_ws_bytes(int B, int n) {
  const size_t N2 = (size_t)n * n;
  const size_t nb = (N2 + GCG_PTS - 1) / GCG_PTS;
  return (4 * B * N2 + 4 * (size_t)B * nb) * sizeof(double) + 2 * (size_t)B * sizeof(int) + 64 +
         coop_ctl_bytes(B, n) + (2 * B * N2 + 1) * sizeof(double);   // + the cooperative CG's s edges
}
// past carve()'s last array (iters), 8-byte aligned
static unsigned long long* coop_ctl(void* ws, int B, int n) {
  const uintptr_t end = reinterpret_cast<uintptr_t>(carve(ws, B, n).iters + B);
  return reinterpret_cast<unsigned long long*>((end + 7) & ~uintptr_t(7));
}

// points per lane (lanes <= 1024): 4 up to n = 24, 7 up to n = 84 (config #3's 40 and 80: 4 and 15
// waves per problem, 128 VGPRs), 16 up to n = 128 (spills part of its five vectors to scratch)
static int lds_npt(int n) { return n <= 24 ? 4 : (n <= 84 ? 7 : 16); }

// f[b][i][j] = sin(2 pi k1_b x_j) sin(2 pi k2_b y_i) on linspace(0,1,n)  (generate_forcing_term,
// data_generation.py:60-77: meshgrid(x, y) -> X varies along columns, Y along rows)
__global__ void forcing_kernel(const double* __restrict__ k, int B, int n, double* __restrict__ out) {
  const long long total = (long long)B * n * n;
  const double h = n > 1 ? 1.0 / (double)(n - 1) : 0.0;
  const double two_pi = 6.283185307179586;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int j = (int)(e % n);
    const long long t = e / n;
    const int i = (int)(t % n);
    const int b = (int)(t / n);
    // linspace(0,1,n)[j] = j * (1/(n-1)), last point exactly 1 (numpy sets the endpoint)
    const double x = (j == n - 1) ? 1.0 : (double)j * h;
    const double y = (i == n - 1) ? 1.0 : (double)i * h;
    out[e] = sin(two_pi * k[2 * b] * x) * sin(two_pi * k[2 * b + 1] * y);
  }
}

}  // namespace srpde

using namespace srpde;

extern "C" {

int srpde_poisson_lds_max_n(void) { return 128; }

int srpde_forcing_batched(const double* k12, int B, int n, double* out, hipStream_t stream) {
  SRPDE_CHECK_ARG(k12 && out && B > 0 && n >= 2, "srpde_forcing_batched: bad args");
  const long long total = (long long)B * n * n;
  const int blocks = (int)std::min<long long>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(forcing_kernel, dim3(blocks), dim3(256), 0, stream, k12, B, n, out);
  SRPDE_LAUNCH_CHECK("srpde_forcing_batched");
  return 0;
}

size_t srpde_poisson_workspace_size(int B, int n) { return n <= 128 ? 0 : grid_ws_bytes(B, n); }

int srpde_poisson_cg_lds(const double* f, const double* theta, double* u, int B, int n, double rtol, int maxit,
                         int* iters, double* resid, hipStream_t stream) {
  SRPDE_CHECK_ARG(f && theta && u && B > 0 && n >= 2 && n <= 128, "srpde_poisson_cg_lds: bad args (n<=128)");
  if (n == 80) {   // config #3's headline size: the compile-time layout (at 20 / 40 the slab layout's
                   // 320-thread blocks ran 2.3x / 1.2x slower than the generic kernel's 128 / 448)
    hipLaunchKernelGGL((cg_lds_n_kernel<80, 960>), dim3(B), dim3(960), 0, stream, f, theta, u, rtol, maxit, iters,
                       resid);
    SRPDE_LAUNCH_CHECK("srpde_poisson_cg_lds");
    return 0;
  }
  const int npt = lds_npt(n);
  int T = ceil_div((long long)n * n, npt);
  T = (T + 63) / 64 * 64;
  SRPDE_CHECK_ARG(T <= CG_MAXT, "srpde_poisson_cg_lds: n too large");
  const size_t lds = ((size_t)(n + 2) * (n + 2) + 64) * sizeof(double);
  switch (npt) {
    case 4: hipLaunchKernelGGL(cg_lds_kernel<4>, dim3(B), dim3(T), lds, stream, f, theta, u, n, rtol, maxit, iters, resid); break;
    case 7: hipLaunchKernelGGL(cg_lds_kernel<7>, dim3(B), dim3(T), lds, stream, f, theta, u, n, rtol, maxit, iters, resid); break;
    default: hipLaunchKernelGGL(cg_lds_kernel<16>, dim3(B), dim3(T), lds, stream, f, theta, u, n, rtol, maxit, iters, resid); break;
  }
  SRPDE_LAUNCH_CHECK("srpde_poisson_cg_lds");
  return 0;
}

int srpde_poisson_cg_grid_init(const double* f, const double* theta, int B, int n, void* ws, size_t ws_bytes,
                               hipStream_t stream) {
  SRPDE_CHECK_ARG(f && theta && ws && B > 0 && n >= 2, "srpde_poisson_cg_grid_init: bad args");
  if (ws_bytes < grid_ws_bytes(B, n)) { set_error("srpde_poisson_cg_grid_init: workspace too small"); return kErrWorkspace; }
  GridCG g = carve(ws, B, n);
  hipLaunchKernelGGL(gcg_init_kernel, dim3(g.nb, B), dim3(GCG_T), 0, stream, f, theta, g);
  hipLaunchKernelGGL(gcg_copy_bb_kernel, dim3(1, B), dim3(256), 0, stream, g);
  SRPDE_LAUNCH_CHECK("srpde_poisson_cg_grid_init");
  return 0;
}

int srpde_poisson_cg_grid_iterate(int B, int n, double rtol, int k_begin, int k_count, int maxit, void* ws,
                                  size_t ws_bytes, hipStream_t stream) {
  SRPDE_CHECK_ARG(ws && ws_bytes >= grid_ws_bytes(B, n), "srpde_poisson_cg_grid_iterate: bad workspace");
  GridCG g = carve(ws, B, n);
  g.rtol = rtol;
  for (int k = k_begin; k < k_begin + k_count; ++k) {
    hipLaunchKernelGGL(gcg_a_kernel, dim3(g.nb, B), dim3(GCG_T), 0, stream, g, k, maxit);
    hipLaunchKernelGGL(gcg_b_kernel, dim3(g.nb, B), dim3(GCG_T), 0, stream, g, k);
  }
  SRPDE_LAUNCH_CHECK("srpde_poisson_cg_grid_iterate");
  return 0;
}

// byte offset of the int32 done-flag vector [B] inside the workspace: lets the host poll convergence
size_t srpde_poisson_cg_grid_done_offset(int B, int n) {
  return (size_t)(reinterpret_cast<char*>(carve(nullptr, B, n).done) - static_cast<char*>(nullptr));
}

int srpde_poisson_cg_grid_finish(double* u, int* iters, int B, int n, int maxit, void* ws, size_t ws_bytes,
                                 hipStream_t stream) {
  SRPDE_CHECK_ARG(u && ws && ws_bytes >= grid_ws_bytes(B, n), "srpde_poisson_cg_grid_finish: bad args");
  GridCG g = carve(ws, B, n);
  const int nbx = std::min(ceil_div((long long)n * n, 256), 1024);
  hipLaunchKernelGGL(gcg_finish_kernel, dim3(nbx, B), dim3(256), 0, stream, g, u, iters, maxit);
  SRPDE_LAUNCH_CHECK("srpde_poisson_cg_grid_finish");
  return 0;
}

static const void* coop_kernel(int npt) {
  switch (npt) {
    case 2: return reinterpret_cast<const void*>(&gcg_coop_kernel<2>);
    case 4: return reinterpret_cast<const void*>(&gcg_coop_kernel<4>);
    default: return reinterpret_cast<const void*>(&gcg_coop_kernel<8>);
  }
}

// co-resident blocks of gcg_coop_kernel<npt> at this n on this device (0: no cooperative launch), cached per
// (device, npt, LDS bytes): a solve asks up to six times
static int coop_capacity(int npt, int n) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  const size_t lds = gcc_lds_bytes(npt, n);
  static std::mutex mu;
  static std::map<std::tuple<int, int, size_t>, int> cache;
  const auto key = std::make_tuple(dev, npt, lds);
  {
    std::lock_guard<std::mutex> lk(mu);
    const auto it = cache.find(key);
    if (it != cache.end()) return it->second;
  }
  int cus = 0, per = 0, coop = 0;
  (void)hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, coop_kernel(npt), GCC_T, lds) != hipSuccess) return 0;
  const int cap = coop ? per * cus : 0;
  std::lock_guard<std::mutex> lk(mu);
  cache[key] = cap;
  return cap;
}

static int coop_blocks(int npt, int n) { return (int)ceil_div((long long)n * n, (long long)GCC_T * npt); }
static int coop_per_launch(int npt, int n) {
  if (2 * n > GCC_HQ * GCC_T || n > GCC_T * npt) return 0;   // halo: the adjacent blocks' rows, <= 2 points per thread
  const int cap = coop_capacity(npt, n), nb = coop_blocks(npt, n);
  return nb <= cap ? cap / nb : 0;
}

// Problems per cooperative launch at this n with the largest blocks (0: one problem does not fit the
// co-resident grid)
int srpde_poisson_coop_problems(int n) { return coop_per_launch(8, n); }

// the whole grid CG of problems [b0, b0 + cnt) in one cooperative launch of gcg_coop_kernel<npt>
// (workspace carved for B: the polled CG's 2048-point partial arrays hold the larger blocks' too)
static int coop_solve(const double* f, const double* theta, double* u, int* iters, int b0, int cnt, int B, int n,
                      int npt, double rtol, int maxit, void* ws, hipStream_t stream, bool start_aborted) {
  const GridCG c = carve(ws, B, n);
  const size_t N2 = (size_t)n * n;
  const int nb = coop_blocks(npt, n);
  GridCoop g;
  // edge values by parity in the polled CG's x / r / p0 / p1 arrays and two more past the ctl words;
  // the partials in its four [B][nb] arrays
  unsigned long long* ctl_all = coop_ctl(ws, B, n);
  double* extra = reinterpret_cast<double*>(reinterpret_cast<char*>(ctl_all) + coop_ctl_bytes(B, n));
  g.er[0] = c.x + b0 * N2; g.er[1] = c.r + b0 * N2;
  g.ew[0] = c.p0 + b0 * N2; g.ew[1] = c.p1 + b0 * N2;
  g.es[0] = extra + b0 * N2; g.es[1] = extra + B * N2 + b0 * N2;
  g.gp[0] = c.rrp0 + (size_t)b0 * nb; g.gp[1] = c.rrp1 + (size_t)b0 * nb;
  g.dp[0] = c.pqp + (size_t)b0 * nb; g.dp[1] = c.bbp + (size_t)b0 * nb;
  g.n = n; g.nb = nb; g.B = cnt; g.rtol = rtol;
  g.ngrp = ceil_div((long long)cnt * nb, COOP_GRP);
  g.bar = ctl_all;
  g.ctl = reinterpret_cast<unsigned*>(g.bar + 1 + g.ngrp);
  hipError_t e = hipMemsetAsync(g.bar, 0, (g.ngrp + 2) * sizeof(unsigned long long), stream);
  if (e == hipSuccess && start_aborted)
    e = hipMemsetAsync(g.ctl + 1, 0x01, 1, stream);
  if (e != hipSuccess) { set_error("srpde_poisson_cg_batched: memset: %s", hipGetErrorString(e)); return (int)e; }
  const double* fb = f + b0 * N2;
  const double* tb = theta + b0 * N2;
  double* ub = u + b0 * N2;
  int* ib = iters ? iters + b0 : nullptr;
  void* args[] = {&fb, &tb, &ub, &ib, &g, &maxit};
  e = hipLaunchCooperativeKernel(coop_kernel(npt), dim3(cnt * nb), dim3(GCC_T), args, gcc_lds_bytes(npt, n), stream);
  if (e != hipSuccess) {
    set_error("srpde_poisson_cg_batched: cooperative launch failed: %s", hipGetErrorString(e));
    return (int)e;
  }
  return 0;
}

// One entry for any n (SURVEY 8(b)'s srpde_poisson_cg_batched), stream-ordered: n <= 128 is one
// launch of the LDS-resident CG; n > 128 runs the grid CG as cooperative launches (one per group of
// srpde_poisson_coop_problems(n) problems), whose grid barriers replace the launch boundaries and
// whose device-side convergence count ends the loop -- nothing returns to the host.  Only a single
// problem too large for the co-resident grid (n > 1024: the halo bound) still runs the launch-per-iteration
// grid CG polled from the host every 128 iterations (that case synchronises `stream`).
// ws: srpde_poisson_workspace_size.
int srpde_poisson_cg_batched(const double* f, const double* theta, double* u, int B, int n, double rtol, int maxit,
                             int* iters_out, void* workspace, size_t ws_bytes, hipStream_t stream) {
  SRPDE_CHECK_ARG(f && theta && u && B > 0 && n >= 2 && maxit >= 0, "srpde_poisson_cg_batched: bad args");
  // rtol < 0: the test hook (|rtol| the tolerance) -- every cooperative launch starts with its abort word set
  const bool start_aborted = rtol < 0;
  rtol = fabs(rtol);
  if (n <= srpde_poisson_lds_max_n())
    return srpde_poisson_cg_lds(f, theta, u, B, n, rtol, maxit, iters_out, nullptr, stream);
  SRPDE_CHECK_ARG(workspace && ws_bytes >= grid_ws_bytes(B, n), "srpde_poisson_cg_batched: workspace too small");
  // Block size: every problem in one launch first; then the smallest blocks that keep the grid to at
  // most half the co-resident capacity -- fewer points per CU against a barrier over more arrivals
  // (per iteration, one problem: 640^2 12.0 / 9.4 / 9.9 us at 2048 / 4096 / 8192-point blocks,
  // 160^2 7.0 / 7.5 / 9.0 us; profiles/r04q_poisson_npt.txt); else the largest blocks (fewest launches)
  int npt = 8;
  for (int pass = 0; pass < 2 && npt == 8; ++pass)
    for (int c : {2, 4}) {
      const int per = coop_per_launch(c, n);
      if (per >= B && (pass == 1 || 2LL * B * coop_blocks(c, n) <= (long long)per * coop_blocks(c, n))) {
        npt = c;
        break;
      }
    }
  const int per = coop_per_launch(npt, n);
  if (per > 0) {
    for (int b0 = 0; b0 < B; b0 += per) {
      const int rc = coop_solve(f, theta, u, iters_out, b0, std::min(per, B - b0), B, n, npt, rtol, maxit, workspace,
                                stream, start_aborted);
      if (rc != 0) return rc;
    }
    return 0;
  }
  constexpr int kCheckEvery = 128;
  int rc = srpde_poisson_cg_grid_init(f, theta, B, n, workspace, ws_bytes, stream);
  if (rc != 0) return rc;
  const int* done_dev = reinterpret_cast<const int*>(static_cast<const char*>(workspace) +
                                                     srpde_poisson_cg_grid_done_offset(B, n));
  std::vector<int> done(B);
  for (int k = 0; k < maxit + 1;) {
    const int cnt = std::min(kCheckEvery, maxit + 1 - k);
    rc = srpde_poisson_cg_grid_iterate(B, n, rtol, k, cnt, maxit, workspace, ws_bytes, stream);
    if (rc != 0) return rc;
    k += cnt;
    hipError_t e = hipMemcpyAsync(done.data(), done_dev, sizeof(int) * B, hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    if (e != hipSuccess) {
      set_error("srpde_poisson_cg_batched: convergence poll failed: %s", hipGetErrorString(e));
      return (int)e;
    }
    if (std::all_of(done.begin(), done.end(), [](int d) { return d != 0; })) break;
  }
  return srpde_poisson_cg_grid_finish(u, iters_out, B, n, maxit, workspace, ws_bytes, stream);
}

}  // extern "C"
