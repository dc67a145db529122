// Row-sharded conjugate gradient for ONE large Poisson problem spread over several ranks
// (cascade row: the 640^2 ground-truth solve of solve_multi_resolution,
// src/resolution_comparison.py:62-73 -> PoissonSolver.solve_poisson, src/data_generation.py:79-104).
//
// Same system and stencil as the grid CG of poisson.hip ((-L) u = -f/theta, 5-point, zero ghost
// ring, h = 1/(n-1)); rank `rank` of `world` owns the contiguous rows [row0, row0 + nloc).  An
// iteration is two launches and two all-gathers, both issued by the caller between the launches:
//
//   A_k: rr_k = sum over ranks of the gathered <r,r> partials (rank order: every rank gets the same
//        bits), beta = rr_k / rr_{k-1}; p_k = r + beta p_{k-1} on the rank's rows, the rows just
//        above / below come from the neighbours' gathered boundary rows of r and p_{k-1};
//        q = A p_k, <p_k, q> of the rank's rows -> spq[0]
//   all-gather spq -> gpq[world]
//   B_k: alpha = rr_k / sum(gpq); x += alpha p_k; r -= alpha q; <r,r> -> send[0], and the rank's
//        first / last rows of r and p_k -> send[1 .. 4n]
//   all-gather send -> gath[world][4n + 1]
//
// Convergence (rr_k <= rtol^2 * rr_0, or k = maxit) is decided inside A_k from the gathered values,
// identically on every rank; a sticky `done` word then turns later launches into no-ops, so the
// host polls it only every few dozen iterations.  Block sums finish in the last block to arrive
// (atomic ticket), in block order: deterministic.  Tested at world 1 and 2 against spsolve
// (tests/test_gpu_poisson_rows.py).
#include "common.h"

namespace srpde {

constexpr int PR_T = 256, PR_NPT = 4, PR_PTS = PR_T * PR_NPT;

struct RowsCG {
  double *x, *r, *p0, *p1, *q;   // [nloc][n]
  double* part;                  // [nb] block partials
  unsigned* ticket;              // last-block counter
  double* st;                    // [0] rr of the last iteration (written by B), [1] rr_0
  int* flag;                     // [0] done, [1] iterations
  int n, nloc, nb;
};

static RowsCG rows_carve(void* ws, int n, int nloc) {
  RowsCG g;
  const size_t N = (size_t)n * nloc;
  g.n = n; g.nloc = nloc; g.nb = (int)((N + PR_PTS - 1) / PR_PTS);
  double* d = static_cast<double*>(ws);
  g.x = d; d += N;
  g.r = d; d += N;
  g.p0 = d; d += N;
  g.p1 = d; d += N;
  g.q = d; d += N;
  g.part = d; d += g.nb;
  g.st = d; d += 2;
  g.ticket = reinterpret_cast<unsigned*>(d);
  g.flag = reinterpret_cast<int*>(d) + 1;
  return g;
}

static size_t rows_ws_bytes(int n, int nloc) {
  const size_t N = (size_t)n * nloc, nb = (N + PR_PTS - 1) / PR_PTS;
  return (5 * N + nb + 2) * sizeof(double) + 4 * sizeof(int) + 64;
}

// sum of v over the block, returned to every thread (fixed order)
__device__ __forceinline__ double rows_block_sum(double v, double* sh) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  double t = 0.0;
  for (int k = 0; k < PR_T / 64; ++k) t += sh[k];
  __syncthreads();
  return t;
}

// block partial -> part[block]; the last block to arrive sums part[] in block order into *out
__device__ __forceinline__ void rows_finish_sum(const RowsCG& g, double v, double* sh, double* out) {
  __shared__ bool last;
  const double s = rows_block_sum(v, sh);
  if (threadIdx.x == 0) {
    g.part[blockIdx.x] = s;
    __threadfence();
    last = atomicAdd(g.ticket, 1u) == (unsigned)(gridDim.x - 1);
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  // every thread of the last block loads a strided share (L1-bypassing), then a fixed-order block sum
  double t = 0.0;
  for (int b = threadIdx.x; b < (int)gridDim.x; b += PR_T) t += *reinterpret_cast<volatile const double*>(g.part + b);
  t = rows_block_sum(t, sh);
  if (threadIdx.x == 0) {
    *out = t;
    *g.ticket = 0u;
  }
}

__global__ __launch_bounds__(PR_T) void rows_init_kernel(const double* __restrict__ f, const double* __restrict__ theta,
                                                         RowsCG g, double* __restrict__ send) {
  __shared__ double sh[PR_T / 64];
  const int n = g.n, N = n * g.nloc;
  double s = 0.0;
  for (int k = 0; k < PR_NPT; ++k) {
    const int i = blockIdx.x * PR_PTS + k * PR_T + threadIdx.x;
    if (i < N) {
      const double rv = -f[i] / theta[i];
      g.x[i] = 0.0; g.r[i] = rv; g.p0[i] = 0.0; g.p1[i] = 0.0; g.q[i] = 0.0;
      s += rv * rv;
      const int yl = i / n, xx = i - yl * n;
      if (yl == 0) { send[1 + xx] = rv; send[1 + 2 * n + xx] = 0.0; }
      if (yl == g.nloc - 1) { send[1 + n + xx] = rv; send[1 + 3 * n + xx] = 0.0; }
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) { g.flag[0] = 0; g.flag[1] = 0; }
  rows_finish_sum(g, s, sh, send);
}

__global__ __launch_bounds__(PR_T) void rows_a_kernel(RowsCG g, int row0, int rank, int world,
                                                      const double* __restrict__ gath, int k, int maxit, double rtol,
                                                      double* __restrict__ spq) {
  __shared__ double sh[PR_T / 64];
  if (g.flag[0]) return;
  const int n = g.n, N = n * g.nloc, stride = 4 * n + 1;
  double rr = 0.0;
  for (int w = 0; w < world; ++w) rr += gath[(size_t)w * stride];
  const double rr0 = k == 0 ? rr : g.st[1];
  if (rr <= rtol * rtol * rr0 || k >= maxit) {
    if (blockIdx.x == 0 && threadIdx.x == 0) { g.flag[0] = 1; g.flag[1] = k; }
    return;
  }
  const double beta = k == 0 ? 0.0 : rr / g.st[0];
  const double* po = (k & 1) ? g.p1 : g.p0;
  double* pn = (k & 1) ? g.p0 : g.p1;
  // neighbours' boundary rows: the rank above's last rows, the rank below's first rows
  const double* up = rank > 0 ? gath + (size_t)(rank - 1) * stride : nullptr;
  const double* dn = rank + 1 < world ? gath + (size_t)(rank + 1) * stride : nullptr;
  const double inv_h2 = (double)(n - 1) * (double)(n - 1);
  double s = 0.0;
  for (int kk = 0; kk < PR_NPT; ++kk) {
    const int i = blockIdx.x * PR_PTS + kk * PR_T + threadIdx.x;
    if (i < N) {
      const int yl = i / n, xx = i - yl * n, y = row0 + yl;
      auto pv = [&](int j) { return g.r[j] + beta * po[j]; };
      const double pc = pv(i);
      double nb = 0.0;
      if (xx > 0) nb += pv(i - 1);
      if (xx < n - 1) nb += pv(i + 1);
      if (y > 0) nb += yl > 0 ? pv(i - n) : up[1 + n + xx] + beta * up[1 + 3 * n + xx];
      if (y < n - 1) nb += yl < g.nloc - 1 ? pv(i + n) : dn[1 + xx] + beta * dn[1 + 2 * n + xx];
      const double qv = (4.0 * pc - nb) * inv_h2;
      pn[i] = pc;
      g.q[i] = qv;
      s += pc * qv;
    }
  }
  rows_finish_sum(g, s, sh, spq);
}

// B_k recomputes rr_k from the same gathered values A_k used (gath is rewritten only after B_k)
// and leaves it in st[0] for A_{k+1}'s beta (st[1] = rr_0 at k = 0): A_k has finished reading st
// (stream order), and no block of B_k reads it.
__global__ __launch_bounds__(PR_T) void rows_b_kernel(RowsCG g, int world, const double* __restrict__ gath,
                                                      const double* __restrict__ gpq, int k, double* __restrict__ send) {
  __shared__ double sh[PR_T / 64];
  if (g.flag[0]) return;
  const int n = g.n, N = n * g.nloc, stride = 4 * n + 1;
  double rr = 0.0, pq = 0.0;
  for (int w = 0; w < world; ++w) rr += gath[(size_t)w * stride];
  for (int w = 0; w < world; ++w) pq += gpq[w];
  const double alpha = rr / pq;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    g.st[0] = rr;
    if (k == 0) g.st[1] = rr;
  }
  const double* pn = (k & 1) ? g.p0 : g.p1;
  double s = 0.0;
  for (int kk = 0; kk < PR_NPT; ++kk) {
    const int i = blockIdx.x * PR_PTS + kk * PR_T + threadIdx.x;
    if (i < N) {
      const double pc = pn[i];
      g.x[i] += alpha * pc;
      const double rn = g.r[i] - alpha * g.q[i];
      g.r[i] = rn;
      s += rn * rn;
      const int yl = i / n, xx = i - yl * n;
      if (yl == 0) { send[1 + xx] = rn; send[1 + 2 * n + xx] = pc; }
      if (yl == g.nloc - 1) { send[1 + n + xx] = rn; send[1 + 3 * n + xx] = pc; }
    }
  }
  rows_finish_sum(g, s, sh, send);
}

__global__ void rows_finish_kernel(RowsCG g, double* __restrict__ u, int* __restrict__ iters, int maxit) {
  const int N = g.n * g.nloc;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < N; i += gridDim.x * blockDim.x) u[i] = g.x[i];
  if (blockIdx.x == 0 && threadIdx.x == 0 && iters) *iters = g.flag[0] ? g.flag[1] : maxit;
}

}  // namespace srpde

using namespace srpde;

extern "C" {

size_t srpde_poisson_rows_workspace_size(int n, int nloc) { return n > 0 && nloc > 0 ? rows_ws_bytes(n, nloc) : 0; }

size_t srpde_poisson_rows_done_offset(int n, int nloc) {
  const size_t N = (size_t)n * nloc, nb = (N + PR_PTS - 1) / PR_PTS;
  return (5 * N + nb + 2) * sizeof(double) + sizeof(int);
}

int srpde_poisson_rows_init(const double* f, const double* theta, int n, int nloc, void* ws, size_t ws_bytes,
                            double* send, hipStream_t stream) {
  SRPDE_CHECK_ARG(f && theta && ws && send && n >= 2 && nloc >= 1 && nloc <= n, "srpde_poisson_rows_init: bad args");
  if (ws_bytes < rows_ws_bytes(n, nloc)) { set_error("srpde_poisson_rows_init: workspace too small"); return kErrWorkspace; }
  RowsCG g = rows_carve(ws, n, nloc);
  (void)hipMemsetAsync(g.ticket, 0, sizeof(unsigned), stream);
  hipLaunchKernelGGL(rows_init_kernel, dim3(g.nb), dim3(PR_T), 0, stream, f, theta, g, send);
  SRPDE_LAUNCH_CHECK("srpde_poisson_rows_init");
  return 0;
}

int srpde_poisson_rows_iter_a(int n, int nloc, int row0, int rank, int world, const double* gath, int k, int maxit,
                              double rtol, void* ws, size_t ws_bytes, double* spq, hipStream_t stream) {
  SRPDE_CHECK_ARG(ws && gath && spq && n >= 2 && nloc >= 1 && world >= 1 && rank >= 0 && rank < world &&
                      row0 >= 0 && row0 + nloc <= n && k >= 0,
                  "srpde_poisson_rows_iter_a: bad args");
  SRPDE_CHECK_ARG((rank > 0) == (row0 > 0) && (rank + 1 < world) == (row0 + nloc < n),
                  "srpde_poisson_rows_iter_a: rows must tile [0, n) in rank order");
  if (ws_bytes < rows_ws_bytes(n, nloc)) { set_error("srpde_poisson_rows_iter_a: workspace too small"); return kErrWorkspace; }
  RowsCG g = rows_carve(ws, n, nloc);
  hipLaunchKernelGGL(rows_a_kernel, dim3(g.nb), dim3(PR_T), 0, stream, g, row0, rank, world, gath, k, maxit, rtol, spq);
  SRPDE_LAUNCH_CHECK("srpde_poisson_rows_iter_a");
  return 0;
}

int srpde_poisson_rows_iter_b(int n, int nloc, int world, const double* gath, const double* gpq, int k, void* ws,
                              size_t ws_bytes, double* send, hipStream_t stream) {
  SRPDE_CHECK_ARG(ws && gath && gpq && send && n >= 2 && nloc >= 1 && world >= 1 && k >= 0,
                  "srpde_poisson_rows_iter_b: bad args");
  if (ws_bytes < rows_ws_bytes(n, nloc)) { set_error("srpde_poisson_rows_iter_b: workspace too small"); return kErrWorkspace; }
  RowsCG g = rows_carve(ws, n, nloc);
  hipLaunchKernelGGL(rows_b_kernel, dim3(g.nb), dim3(PR_T), 0, stream, g, world, gath, gpq, k, send);
  SRPDE_LAUNCH_CHECK("srpde_poisson_rows_iter_b");
  return 0;
}

int srpde_poisson_rows_finish(double* u, int* iters, int n, int nloc, int maxit, void* ws, size_t ws_bytes,
                              hipStream_t stream) {
  SRPDE_CHECK_ARG(u && ws && n >= 2 && nloc >= 1, "srpde_poisson_rows_finish: bad args");
  if (ws_bytes < rows_ws_bytes(n, nloc)) { set_error("srpde_poisson_rows_finish: workspace too small"); return kErrWorkspace; }
  RowsCG g = rows_carve(ws, n, nloc);
  hipLaunchKernelGGL(rows_finish_kernel, dim3(std::min(g.nb * 4, 1024)), dim3(256), 0, stream, g, u, iters, maxit);
  SRPDE_LAUNCH_CHECK("srpde_poisson_rows_finish");
  return 0;
}

}  // extern "C"
