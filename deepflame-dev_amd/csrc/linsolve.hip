// linsolve.hip -- Krylov solvers on the assembled LDU systems (replaces the AmgX path, reference
// src_gpu/AmgXSolver.cu:184-340 and dfMatrixDataBase.cu:166-177, and the per-matrix ldu_to_csr
// gathers dfMatrixOpBase.cu:2276-2352 / dfUEqn.cu:836-894).
//
// Storage: a static ELL gather built once from the mesh, [W][C] (coalesced): per cell W coupling
// entries in OpenFOAM's sequential order -- faces where the cell is neighbour (lower), faces it owns
// (upper), then its coupled boundary slots (cyclic partner cell, or processor halo entry C + h). Per
// solve one pass folds lower/upper/-boundaryCoeffs into ELL values and diag + internalCoeffs into the
// diagonal (fvMatrix::addBoundaryDiag / addBoundarySource, the work ldu_to_csr does in the reference).
// Systems sharing a sparsity pattern run as one batch (grid.y = system): the 3 U components, and all
// non-inert species of the Y equation (independent matrices; the reference's sequential species loop
// becomes a batch).
//
// Iterations have no single-block "finalise" kernels: every kernel that needs a global dot product
// reduces the previous kernel's per-block partials itself in its prologue (fixed order, identical in
// every block, so bitwise deterministic), and block 0 records the scalars for the host. Across ranks
// the per-rank sums are all-gathered (RCCL) and summed in rank order. Jacobi preconditioning on
// diag + internalCoeffs; convergence AmgX RELATIVE_INI L2 (||r|| <= tol ||r0||), per system; the host
// reads the per-system state every `check` iterations (inactive systems turn every kernel into a no-op).
#include "dfmi_ctx.h"
#include <climits>
#include <cmath>
#include <cstdlib>

namespace dfmi {
namespace {

constexpr int TPB = 256;
constexpr int NW = TPB / 64;
constexpr int MAX_BLOCKS = 2048;
// blocks of the even-odd half-row passes: measured 256 / 512 / 768 / 1024 / 2048 / 3072 / 4096
// -> 42.8 / 34.7 / 36.7 / 32.8 / 35.1 / 47.7 / 45.0 us per Schur application (the partial sums every consumer
// block re-sums grow with the grid; fewer blocks leave too few waves)
constexpr int EO_BLOCKS = 1024;
inline int eo_max_blocks() { return EO_BLOCKS; }
// blocks of the PCG kernels (1024 / 1536 / 2048: 43.2 / 38.9 / 37.8 us per k_cg_spmv, round 4)
inline int cg_max_blocks() { return MAX_BLOCKS; }
constexpr int PAD = INT_MIN;
constexpr int NSCAL = 16;

static_assert(TPB == RED_TPB, "the fixed-order reductions (dfmi_common.h red_sum) assume 256-thread blocks");

// block partial of NV values -> partial[(s * nblk + blockIdx.x) * NV + k]
// Row sets of the halo-overlapped SpMVs (multi-rank, DFMI_HALO_OVERLAP=1): part 1 = the rows without a
// processor column (they run while the halo exchange is in flight on the comm stream), part 2 = the
// listed boundary rows (after it). Each part writes its block partials into its own half of a
// [system][2 nblk] layout, which the consumer reduces in fixed order. part 0 = every row, one pass.
struct RowSet {
  int part = 0;
  const int8_t* flag = nullptr;   // [C] 1: the row has a processor column
  const int* list = nullptr;      // the boundary rows
  int nb = 0;
};
__device__ __forceinline__ int rows_begin() { return xcd_block() * blockDim.x + threadIdx.x; }
template <class F> __device__ __forceinline__ void for_rows(long C, const RowSet& rs, F&& f) {
  // one loop (the body is instantiated once: two loops measured +19 % on k_bcg_spmv2)
  const int stride = gridDim.x * blockDim.x;
  const int n = rs.part == 2 ? rs.nb : (int)C;
  for (int k = rows_begin(); k < n; k += stride) {
    const int c = rs.part == 2 ? rs.list[k] : k;
    if (rs.part == 1 && rs.flag[c]) continue;
    f(c);
  }
}

template <int NV> __device__ __forceinline__ void block_partials(double (&v)[NV], double* partial, int s,
                                                                const RowSet& rs = RowSet{}) {
  __shared__ double sh[NW][NV];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) { const double t = wave_sum(v[k]); if (lane == 0) sh[wid][k] = t; }
  __syncthreads();
  if (threadIdx.x < NV) {
    double a = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) a += sh[w][threadIdx.x];
    const int gt = rs.part ? 2 * gridDim.x : gridDim.x, bo = rs.part == 2 ? gridDim.x : 0;
    partial[((long)s * gt + bo + blockIdx.x) * NV + threadIdx.x] = a;
  }
}

template <int NV> __global__ void k_red_local(const double* partial, int nblk, double* out) {
  const int s = blockIdx.x;
  double v[NV];
  red_sum<NV>(Red{partial, nblk, NV, (long)nblk * NV}, s, v);
  if (threadIdx.x == 0)
#pragma unroll
    for (int k = 0; k < NV; ++k) out[s * NV + k] = v[k];
}

__device__ __forceinline__ bool leader() { return blockIdx.x == 0 && threadIdx.x == 0; }

// y = dS x + sum_k val[k] x[col[k]]  (lduMatrix::Amul + updateMatrixInterfaces, same order)
template <int WT> __device__ __forceinline__ double ell_mv(int W_, long C, const ColView& col, const int* sh,
                                                            const double* __restrict__ val, double d,
                                                            const double* __restrict__ xv, int c) {
  const int W = WT > 0 ? WT : W_;
  const int rb = col.row(c);
  double y = d * xv[c];
#pragma unroll
  for (int k = 0; k < W; ++k) y += val[k * C + c] * xv[col.get(sh, rb, C, k, c)];
  return y;
}

struct Sys {
  const double *lower, *upper, *diag, *source, *ic, *bc;
  long lstride, ustride, dstride, sstride, bstride;
  double* x; long xstride;
};

// per system: ELL values, dS = diag + sum internalCoeffs, rhs = source + non-coupled boundaryCoeffs
// (fvMatrix::addBoundaryDiag / addBoundarySource(source, false)), slot order as the sequential code
// vshared: the systems share one operator (U's components: one LDU, and the coupled-slot coefficients of
// translational cyclic / processor patches do not depend on the component), so only system 0 writes val;
// 2: no values at all (a PCG that reads the operator face-wise and reuses the V-cycle built earlier)
__global__ void k_ell_build(MeshView m, const int8_t* __restrict__ ty, Sys q, const int* __restrict__ sys_map, int W,
                            const int* __restrict__ esrc, long Ce, double* __restrict__ val, double* __restrict__ dS,
                            double* __restrict__ rhs, int vshared = 0, const int* __restrict__ eopos = nullptr) {
  const int s = blockIdx.y;
  const int ms = sys_map ? sys_map[s] : s;
  const long C = m.C;
  const double* L = q.lower + ms * q.lstride;
  const double* U = q.upper + ms * q.ustride;
  const double* ic = q.ic + ms * q.bstride;
  const double* bc = q.bc + ms * q.bstride;
  double* vs = val + (long)s * W * C;
  const bool wv = vshared == 0 || (vshared == 1 && s == 0);
  for (int c = xcd_block() * blockDim.x + threadIdx.x; c < m.C; c += gridDim.x * blockDim.x) {
    const int pc = eopos ? eopos[c] : c;   // the row of c (even-odd layout) or c
    const int cl = ecls_of(m, c);
    for (int k = 0; wv && k < W; ++k) {
      int j, e;
      erow(m, cl, k, c, j, e);
      double v;
      if (e == PAD) v = 0.0;
      else if (e >= 0) v = (e & 1) ? U[e >> 1] : L[e >> 1];
      else v = -bc[-e - 1];
      vs[k * C + pc] = v;
    }
    double d = q.diag[ms * q.dstride + c];
    double r = q.source[ms * q.sstride + c];
    const int e3 = m.cbStart[c + 1];
    for (int k = m.cbStart[c]; k < e3; ++k) {
      const int b = m.cbSlot[k];
      if (ty[b] == EMPTY) continue;
      d += ic[b];
    }
    for (int k = m.cbStart[c]; k < e3; ++k) {
      const int b = m.cbSlot[k];
      const int t = ty[b];
      if (t == EMPTY || bc_coupled(t)) continue;
      r += bc[b];
    }
    dS[s * Ce + pc] = d;
    rhs[s * Ce + pc] = r;
  }
}

// copy the current solution into a work vector (its halo region is filled by the exchange)
__global__ void k_copy_x(long C, long Ce, Sys q, const int* __restrict__ sys_map, double* __restrict__ xw,
                         const int* __restrict__ eopos = nullptr) {
  const int s = blockIdx.y;
  const int ms = sys_map ? sys_map[s] : s;
  for (long c = xcd_block() * (long)blockDim.x + threadIdx.x; c < C; c += (long)gridDim.x * blockDim.x)
    xw[s * Ce + (eopos ? eopos[c] : c)] = q.x[ms * q.xstride + c];
}

// ============================================================== BiCGStab (AmgX PBiCGStab semantics)
// Jacobi-scaled BiCGStab: the iteration runs on D^-1 A x = D^-1 b (D = diag + internalCoeffs), so the
// operator has a unit diagonal, no preconditioned copies of p and s are stored, and the convergence
// test uses the true residual norm ||b - A x|| = ||D r|| (AmgX RELATIVE_INI_CORE, L2). Four kernels
// per iteration: v = A p, s = r - alpha v, t = A s, and one fused update x += alpha p + omega s,
// r = s - omega t, p = r + beta (p - omega v) -- rho_new = r0.r comes from the recurrence
// r0.s - omega r0.t, whose two dot products the previous kernels already reduced, so the next
// direction is formed in the same pass as the solution update.
// scal[s*16 + k]: 0 rho, 1 rho_old, 2 alpha, 3 omega, 4 res0, 5 res, 6 active, 7 iters, 8 rho_new (the
// update kernel writes it, the next SpMV publishes it as rho: no scalar is rewritten by the kernel whose
// other blocks read it)
struct BV { double *dS, *rhs, *r, *r0, *p, *v, *sv, *t, *xw; int vshared; };
constexpr int BCG_VECS = 9;

// y = (A in)_c / D_c = in_c + (sum_k val in_j) / D_c
template <int WT> __device__ __forceinline__ double scaled_mv(int W_, long C, const ColView& col, const int* sh,
                                                              const double* __restrict__ val, double d,
                                                              const double* __restrict__ xv, int c) {
  const int W = WT > 0 ? WT : W_;
  const int rb = col.row(c);
  double o = 0.0;
#pragma unroll
  for (int k = 0; k < W; ++k) o += val[k * C + c] * xv[col.get(sh, rb, C, k, c)];
  return xv[c] + o / d;
}

// r = D^-1 (b - A x); r0 = p = r; partials (||D r||^2, r0.r)
template <int WT>
__global__ void __launch_bounds__(TPB) k_bcg_init(long C, long Ce, int W, ColView col,
                                                  const double* __restrict__ val, BV b, double* partial) {
  const int s = blockIdx.y;
  const double* vs = val + (long)(b.vshared ? 0 : s) * W * C;
  __shared__ int s_ct[CT_MAX];
  col.stage(s_ct);
  double acc[2] = {0.0, 0.0};
  for (int c = xcd_block() * blockDim.x + threadIdx.x; c < C; c += gridDim.x * blockDim.x) {
    const long i = s * Ce + c;
    const double d = b.dS[i];
    const double res = b.rhs[i] - ell_mv<WT>(W, C, col, s_ct, vs, d, b.xw + s * Ce, c);
    const double rr = res / d;
    b.r[i] = rr; b.r0[i] = rr; b.p[i] = rr;
    acc[0] += res * res;
    acc[1] += rr * rr;
  }
  block_partials<2>(acc, partial, s);
}

// prologue: res = ||D r||, rho; convergence; v = D^-1 A p; partial r0.v
template <int WT>
__global__ void __launch_bounds__(TPB) k_bcg_spmv1(long C, long Ce, int W, ColView col,
                                                   const double* __restrict__ val, int it, int max_iter, double tol,
                                                   double abs_tol, Red red, double* scal, BV b, double* partial,
                                                   RowSet rs) {
  const int s = blockIdx.y;
  double* st = scal + s * NSCAL;
  if (it > 0 && st[6] == 0.0) return;   // stopped earlier (uniform per block)
  double v2[2];
  red_sum<2>(red, s, v2);
  const double res = sqrt(v2[0]);
  const double rho = it == 0 ? v2[1] : st[8];   // r0.r: initial, or the previous update's recurrence
  const double res0 = it == 0 ? res : st[4];
  const bool stop = res <= tol * res0 || res <= abs_tol || it >= max_iter || (it > 0 && (rho == 0.0 || st[3] == 0.0));
  if (leader() && rs.part != 2) {
    if (it == 0) st[4] = res;
    st[0] = rho;
    st[5] = res; st[7] = it;
    st[6] = stop ? 0.0 : 1.0;
  }
  if (stop) return;
  const double* vs = val + (long)(b.vshared ? 0 : s) * W * C;
  __shared__ int s_ct[CT_MAX];
  col.stage(s_ct);
  double acc[1] = {0.0};
  for_rows(C, rs, [&](int c) {
    const long i = s * Ce + c;
    const double y = scaled_mv<WT>(W, C, col, s_ct, vs, b.dS[i], b.p + s * Ce, c);
    b.v[i] = y;
    acc[0] += b.r0[i] * y;
  });
  block_partials<1>(acc, partial, s, rs);
}

// multi-rank only: s = r - alpha v into sv, whose processor-boundary values the halo exchange sends
__global__ void __launch_bounds__(TPB) k_bcg_s(long C, long Ce, Red red, double* scal, BV b) {
  const int s = blockIdx.y;
  double* st = scal + s * NSCAL;
  if (st[6] == 0.0) return;
  double v[1];
  red_sum<1>(red, s, v);
  const double alpha = v[0] != 0.0 ? st[0] / v[0] : 0.0;
  for (int c = xcd_block() * blockDim.x + threadIdx.x; c < C; c += gridDim.x * blockDim.x) {
    const long i = s * Ce + c;
    b.sv[i] = b.r[i] - alpha * b.v[i];
  }
}

// prologue: alpha = rho / (r0.v). s = r - alpha v is formed on the fly (own cell and every neighbour:
// the gathers of r and v hit the same lines as the own-cell reads of other threads), so no kernel writes
// s and nothing re-reads it; halo entries (processor neighbours, j >= C) read the exchanged copy sv.
// t = D^-1 A s; partials (t.s, t.t, r0.t, r0.s)
template <int WT>
__global__ void __launch_bounds__(TPB) k_bcg_spmv2(long C, long Ce, int W_, ColView col,
                                                   const double* __restrict__ val, Red red, double* scal, BV b,
                                                   double* partial, RowSet rows) {
  const int s = blockIdx.y;
  double* st = scal + s * NSCAL;
  if (st[6] == 0.0) return;   // uniform per block
  double v1[1];
  red_sum<1>(red, s, v1);
  const double alpha = v1[0] != 0.0 ? st[0] / v1[0] : 0.0;
  if (leader() && rows.part != 2) st[2] = alpha;
  const int W = WT > 0 ? WT : W_;
  const double* vs = val + (long)(b.vshared ? 0 : s) * W * C;
  const double* rs = b.r + s * Ce;
  const double* ws = b.v + s * Ce;
  const double* hs = b.sv + s * Ce;
  __shared__ int s_ct[CT_MAX];
  col.stage(s_ct);
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  for_rows(C, rows, [&](int c) {
    const long i = s * Ce + c;
    const double sc = rs[c] - alpha * ws[c];
    const int rb = col.row(c);
    double o = 0.0;
#pragma unroll
    for (int k = 0; k < W; ++k) {
      const int j = col.get(s_ct, rb, C, k, c);
      const double sj = j < C ? rs[j] - alpha * ws[j] : hs[j];
      o += vs[k * C + c] * sj;
    }
    const double y = sc + o / b.dS[i];
    b.t[i] = y;
    const double r0 = b.r0[i];
    acc[0] += y * sc;
    acc[1] += y * y;
    acc[2] += r0 * y;
    acc[3] += r0 * sc;
  });
  block_partials<4>(acc, partial, s, rows);
}

// prologue: omega = (t.s)/(t.t); rho_new = r0.s - omega r0.t; beta = (rho_new / rho)(alpha / omega);
// x += alpha p + omega s; r = s - omega t; p = r + beta (p - omega v); partials (||D r||^2, 0)
__global__ void __launch_bounds__(TPB) k_bcg_xp(long C, long Ce, Red red_t, Sys q, const int* __restrict__ sys_map,
                                                double* scal, BV b, double* partial) {
  const int s = blockIdx.y;
  double* st = scal + s * NSCAL;
  if (st[6] == 0.0) return;
  double tv[4];
  red_sum<4>(red_t, s, tv);
  const double omega = tv[1] != 0.0 ? tv[0] / tv[1] : 0.0;
  const double alpha = st[2], rho = st[0];
  const double rho_new = tv[3] - omega * tv[2];
  const double beta = (rho != 0.0 && omega != 0.0) ? (rho_new / rho) * (alpha / omega) : 0.0;
  if (leader()) { st[3] = omega; st[1] = rho; st[8] = rho_new; }   // st[0] is read by every block of this kernel
  const int ms = sys_map ? sys_map[s] : s;
  double* xv = q.x + ms * q.xstride;
  double acc[2] = {0.0, 0.0};
  for (int c = xcd_block() * blockDim.x + threadIdx.x; c < C; c += gridDim.x * blockDim.x) {
    const long i = s * Ce + c;
    const double pv = b.p[i], vv = b.v[i];
    const double sv = b.r[i] - alpha * vv;   // the s of k_bcg_spmv2, same expression
    xv[c] = xv[c] + alpha * pv + omega * sv;
    const double rr = sv - omega * b.t[i];
    b.r[i] = rr;
    b.p[i] = rr + beta * (pv - omega * vv);
    const double tr = b.dS[i] * rr;
    acc[0] += tr * tr;
  }
  block_partials<2>(acc, partial, s);
}

// convergence record of a solve into host-coherent memory (Poller, below), by one wave (lane = threadIdx.x & 63):
// lane s reads system s (vector loads, vector stores)
__device__ __forceinline__ void poll_post(const double* __restrict__ scal, int nsys, PollRec* rec, long long seq) {
  const int lane = threadIdx.x & 63;
  int act = 0, it = 0;
  for (int s = lane; s < nsys; s += 64) {
    act |= scal[s * NSCAL + 6] != 0.0;
    it = max(it, (int)scal[s * NSCAL + 7]);
  }
  for (int o = 32; o > 0; o >>= 1) { act |= __shfl_xor(act, o, 64); it = max(it, __shfl_xor(it, o, 64)); }
  if (lane == 0) {
    PollRec* r = rec + (seq & 1);
    r->stopped = act ? 0 : 1;
    r->iters = it;
    __hip_atomic_store(&r->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
// ============================================================== even-odd (red-black) reduced BiCGStab
// On a coupling graph that 2-colours (every entry of a row couples the other colour: hex meshes, walled or
// periodic with even cyclic extents) the Jacobi-scaled system splits as
//   [ I     H_eo ] [x_e]   [b_e]       H_eo = D_e^-1 O_eo,  H_oe = D_o^-1 O_oe,  b = D^-1 rhs
//   [ H_oe  I    ] [x_o] = [b_o]
// and BiCGStab runs on the colour-1 Schur complement  S x_o = b_o - H_oe b_e,  S = I - H_oe H_eo  (the
// even-odd preconditioning of lattice QCD's nearest-neighbour solvers); afterwards x_e = b_e - H_eo x_o.
// The full residual of that x is 0 on colour 0 and D_o r_o on colour 1, so AmgX's RELATIVE_INI_CORE test
// on ||b - A x|| (against the full residual of the initial guess) is evaluated exactly on the reduced
// residual. Where the Jacobi-scaled operator's off-diagonal part has spectral radius mu (0.3 - 0.7 on
// these diagonally dominant U / Y / E systems), S's eigenvalues lie in 1 - mu^2 instead of 1 +- mu:
// about half the iterations for about the bytes of one full SpMV per application of S (two half-row
// passes). Rows and vectors are stored colour by colour (Ctx::Ell::eo): colour 0 in [0, ne), colour 1 in
// [ne, C). The colour-0 half of p holds g / w = H_eo p and the colour-0 half of t holds w2 = H_eo s.
// scal: as BiCGStab, plus 9 = the initial guess already met abs_tol (x left untouched).
template <class F> __device__ __forceinline__ void for_half(int n, F&& f) {
  for (int m = xcd_block() * blockDim.x + threadIdx.x; m < n; m += gridDim.x * blockDim.x) f(m);
}

// colour-0 rows: g = (rhs - O x0_o) / D (= b_e - H_eo x0_o, into p's colour-0 half); partial
// ||b - A x0||^2 over these rows
template <int WT>
__global__ void __launch_bounds__(TPB) k_eo_init_e(long C, long Ce, int ne, int W_, ColView col,
                                                   const double* __restrict__ val, BV b, double* partial) {
  const int s = blockIdx.y;
  const int W = WT > 0 ? WT : W_;
  const double* vs = val + (long)(b.vshared ? 0 : s) * W * C;
  const double* xw = b.xw + s * Ce;
  __shared__ int s_ct[CT_MAX];
  col.stage(s_ct);
  double acc[1] = {0.0};
  for_half(ne, [&](int i) {
    const long ii = s * Ce + i;
    const int rb = col.row(i);
    double o = 0.0;
    for_cols<WT>(col, s_ct, rb, C, W, i, [&](int k, int j) { o += vs[k * C + i] * xw[j]; });
    const double d = b.dS[ii], rh = b.rhs[ii];
    b.p[ii] = (rh - o) / d;
    const double res = rh - d * xw[i] - o;
    acc[0] += res * res;
  });
  block_partials<1>(acc, partial, s);
}

// colour-1 rows: ||b - A x0||^2 (the initial guess's own colour-0 values); reduced residual
// r = (rhs - O g) / D - x0_o; r0 = p = r; partials (||b - A x0||^2, ||D r||^2, r0.r)
template <int WT>
__global__ void __launch_bounds__(TPB) k_eo_init_o(long C, long Ce, int ne, int no, int W_, ColView col,
                                                   const double* __restrict__ val, BV b, double* partial) {
  const int s = blockIdx.y;
  const int W = WT > 0 ? WT : W_;
  const double* vs = val + (long)(b.vshared ? 0 : s) * W * C;
  const double* xw = b.xw + s * Ce;
  const double* ps = b.p + s * Ce;
  __shared__ int s_ct[CT_MAX];
  col.stage(s_ct);
  double acc[3] = {0.0, 0.0, 0.0};
  for_half(no, [&](int m) {
    const int i = ne + m;
    const long ii = s * Ce + i;
    const int rb = col.row(i);
    double o1 = 0.0, o2 = 0.0;
    for_cols<WT>(col, s_ct, rb, C, W, i, [&](int k, int j) {
      const double a = vs[k * C + i];
      o1 += a * xw[j];
      o2 += a * ps[j];
    });
    const double d = b.dS[ii], rh = b.rhs[ii], xo = xw[i];
    const double res = rh - d * xo - o1;
    const double r = (rh - o2) / d - xo;
    b.r[ii] = r; b.r0[ii] = r; b.p[ii] = r;
    const double tr = d * r;
    acc[0] += res * res;
    acc[1] += tr * tr;
    acc[2] += r * r;
  });
  block_partials<3>(acc, partial, s);
}

// prologue: res0 (it 0: the full initial residual), res = ||D r||, rho, convergence;
// colour-0 rows: w = H_eo p (p's colour-0 half)
// defer (several ranks, it > 0): ||D r|| rides the next all-gather (k_eo_c's) instead of its own, so the stop test
// moves there; this launch only takes rho (k_eo_xp's) and forms w
template <int WT>
__global__ void __launch_bounds__(TPB) k_eo_a(long C, long Ce, int ne, int W_, ColView col,
                                              const double* __restrict__ val, int it, int max_iter, double tol,
                                              double abs_tol, Red redI, Red redR, double* scal, BV b, int defer = 0) {
  const int s = blockIdx.y;
  double* st = scal + s * NSCAL;
  if (it > 0 && st[6] == 0.0) return;   // stopped earlier (uniform per block)
  if (defer) {
    if (leader()) st[0] = st[8];
  } else {
    double res0, n2, rho;
    if (it == 0) {
      double e[1], o[3];
      red_sum<1>(redI, s, e);
      red_sum<3>(redR, s, o);
      res0 = sqrt(e[0] + o[0]); n2 = o[1]; rho = o[2];
    } else {
      double o[2];
      red_sum<2>(redR, s, o);
      n2 = o[0]; rho = st[8]; res0 = st[4];
    }
    const double res = sqrt(n2);
    const bool keep = it == 0 && (res0 <= abs_tol || res0 == 0.0);
    const bool stop = keep || res <= tol * res0 || res <= abs_tol || it >= max_iter ||
                      (it > 0 && (rho == 0.0 || st[3] == 0.0));
    if (leader()) {
      if (it == 0) { st[4] = res0; st[9] = keep ? 1.0 : 0.0; }
      st[0] = rho;
      st[5] = res; st[7] = it;
      st[6] = stop ? 0.0 : 1.0;
    }
    if (stop) return;
  }
  const int W = WT > 0 ? WT : W_;
  const double* vs = val + (long)(b.vshared ? 0 : s) * W * C;
  double* ps = b.p + s * Ce;
  __shared__ int s_ct[CT_MAX];
  col.stage(s_ct);
  for_half(ne, [&](int i) {
    const int rb = col.row(i);
    double o = 0.0;
    for_cols<WT>(col, s_ct, rb, C, W, i, [&](int k, int j) { o += vs[k * C + i] * ps[j]; });
    ps[i] = o / b.dS[s * Ce + i];
  });
}

// colour-1 rows: v = S p = p - H_oe w; partial r0.v
template <int WT>
__global__ void __launch_bounds__(TPB) k_eo_b(long C, long Ce, int ne, int no, int W_, ColView col,
                                              const double* __restrict__ val, double* scal, BV b, double* partial) {
  const int s = blockIdx.y;
  if (scal[s * NSCAL + 6] == 0.0) return;
  const int W = WT > 0 ? WT : W_;
  const double* vs = val + (long)(b.vshared ? 0 : s) * W * C;
  const double* ps = b.p + s * Ce;
  __shared__ int s_ct[CT_MAX];
  col.stage(s_ct);
  double acc[1] = {0.0};
  for_half(no, [&](int m) {
    const int i = ne + m;
    const long ii = s * Ce + i;
    const int rb = col.row(i);
    const double r0 = b.r0[ii];   // before the store: b.v may alias it as far as the compiler knows
    double o = 0.0;
    for_cols<WT>(col, s_ct, rb, C, W, i, [&](int k, int j) { o += vs[k * C + i] * ps[j]; });
    const double y = ps[i] - o / b.dS[ii];
    b.v[ii] = y;
    acc[0] += r0 * y;
  });
  block_partials<1>(acc, partial, s);
}

// prologue: alpha = rho / (r0.v); colour-0 rows: w2 = H_eo s, s = r - alpha v formed at the neighbours
// defer (k_eo_a's): redV also carries ||D r||^2 of the last update -- the stop test of this iteration runs here
template <int WT>
__global__ void __launch_bounds__(TPB) k_eo_c(long C, long Ce, int ne, int W_, ColView col,
                                              const double* __restrict__ val, Red redV, double* scal, BV b,
                                              int defer = 0, int it = 0, double tol = 0.0, double abs_tol = 0.0) {
  const int s = blockIdx.y;
  double* st = scal + s * NSCAL;
  if (st[6] == 0.0) return;
  double rv[2];
  if (defer) {
    red_sum<2>(redV, s, rv);
    const double res = sqrt(rv[1]);
    const bool stop = res <= tol * st[4] || res <= abs_tol || st[0] == 0.0 || st[3] == 0.0;
    if (leader()) {
      st[5] = res; st[7] = it;
      if (stop) st[6] = 0.0;
    }
    if (stop) return;
  } else {
    double r1[1];
    red_sum<1>(redV, s, r1);
    rv[0] = r1[0];
  }
  const double alpha = rv[0] != 0.0 ? st[0] / rv[0] : 0.0;
  if (leader()) st[2] = alpha;
  const int W = WT > 0 ? WT : W_;
  const double* vs = val + (long)(b.vshared ? 0 : s) * W * C;
  const double* rs = b.r + s * Ce;
  const double* ws = b.v + s * Ce;
  double* ts = b.t + s * Ce;
  __shared__ int s_ct[CT_MAX];
  col.stage(s_ct);
  for_half(ne, [&](int i) {
    const int rb = col.row(i);
    double o = 0.0;
    for_cols<WT>(col, s_ct, rb, C, W, i, [&](int k, int j) { o += vs[k * C + i] * (rs[j] - alpha * ws[j]); });
    ts[i] = o / b.dS[s * Ce + i];
  });
}

// several ranks: this rank's (r0.v, ||D r||^2) per system from k_eo_b's and k_eo_xp's block partials, for one
// all-gather
__global__ void k_red_vr(const double* pV, const double* pR, int nblk, double* out) {
  const int s = blockIdx.x;
  double a[1], c[1];
  red_sum<1>(Red{pV, nblk, 1, (long)nblk}, s, a);
  red_sum<1>(Red{pR, nblk, 2, 2L * nblk}, s, c);
  if (threadIdx.x == 0) { out[2 * s] = a[0]; out[2 * s + 1] = c[0]; }
}

// colour-1 rows: t = S s = s - H_oe w2; partials (t.s, t.t, r0.t, r0.s)
template <int WT>
__global__ void __launch_bounds__(TPB) k_eo_d(long C, long Ce, int ne, int no, int W_, ColView col,
                                              const double* __restrict__ val, double* scal, BV b, double* partial) {
  const int s = blockIdx.y;
  const double* st = scal + s * NSCAL;
  if (st[6] == 0.0) return;
  const double alpha = st[2];
  const int W = WT > 0 ? WT : W_;
  const double* vs = val + (long)(b.vshared ? 0 : s) * W * C;
  double* ts = b.t + s * Ce;
  __shared__ int s_ct[CT_MAX];
  col.stage(s_ct);
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  for_half(no, [&](int m) {
    const int i = ne + m;
    const long ii = s * Ce + i;
    const int rb = col.row(i);
    const double r0 = b.r0[ii];
    double o = 0.0;
    for_cols<WT>(col, s_ct, rb, C, W, i, [&](int k, int j) { o += vs[k * C + i] * ts[j]; });
    const double sc = b.r[ii] - alpha * b.v[ii];
    const double y = sc - o / b.dS[ii];
    ts[i] = y;
    acc[0] += y * sc;
    acc[1] += y * y;
    acc[2] += r0 * y;
    acc[3] += r0 * sc;
  });
  block_partials<4>(acc, partial, s);
}

// colour-1 rows, k_bcg_xp's update on the reduced vectors (x_o in xw's colour-1 half)
// rec != nullptr: wave 0 of block (0, 0) also posts convergence record `seq` (Poller::plan) before anything else --
// the systems' flags and counts it reads were final after k_eo_a, exactly what a k_poll_post after this kernel reads
__global__ void __launch_bounds__(TPB) k_eo_xp(long Ce, int ne, int no, Red red_t, double* scal, BV b,
                                               double* partial, PollRec* rec = nullptr, long long seq = 0) {
  const int s = blockIdx.y;
  if (rec && blockIdx.x == 0 && s == 0 && threadIdx.x < 64) poll_post(scal, gridDim.y, rec, seq);
  double* st = scal + s * NSCAL;
  if (st[6] == 0.0) return;
  double tv[4];
  red_sum<4>(red_t, s, tv);
  const double omega = tv[1] != 0.0 ? tv[0] / tv[1] : 0.0;
  const double alpha = st[2], rho = st[0];
  const double rho_new = tv[3] - omega * tv[2];
  const double beta = (rho != 0.0 && omega != 0.0) ? (rho_new / rho) * (alpha / omega) : 0.0;
  if (leader()) { st[3] = omega; st[1] = rho; st[8] = rho_new; }
  double acc[2] = {0.0, 0.0};
  for_half(no, [&](int m) {
    const long ii = s * Ce + ne + m;
    const double pv = b.p[ii], vv = b.v[ii];
    const double sv = b.r[ii] - alpha * vv;
    b.xw[ii] = b.xw[ii] + alpha * pv + omega * sv;
    const double rr = sv - omega * b.t[ii];
    b.r[ii] = rr;
    b.p[ii] = rr + beta * (pv - omega * vv);
    const double tr = b.dS[ii] * rr;
    acc[0] += tr * tr;
  });
  block_partials<2>(acc, partial, s);
}

// after the iterations: x_o from xw, x_e = (rhs - O x_o) / D, back into the caller's cell order
template <int WT>
__global__ void __launch_bounds__(TPB) k_eo_final(long C, long Ce, int ne, int no, int W_, ColView col,
                                                  const double* __restrict__ val, const double* scal, BV b, Sys q,
                                                  const int* __restrict__ sys_map, const int* __restrict__ eocell) {
  const int s = blockIdx.y;
  if (scal[s * NSCAL + 9] != 0.0) return;   // the initial guess met abs_tol: left as it was
  const int ms = sys_map ? sys_map[s] : s;
  double* xv = q.x + ms * q.xstride;
  const int W = WT > 0 ? WT : W_;
  const double* vs = val + (long)(b.vshared ? 0 : s) * W * C;
  const double* xw = b.xw + s * Ce;
  __shared__ int s_ct[CT_MAX];
  col.stage(s_ct);
  for_half(ne, [&](int i) {
    const int rb = col.row(i);
    double o = 0.0;
    for_cols<WT>(col, s_ct, rb, C, W, i, [&](int k, int j) { o += vs[k * C + i] * xw[j]; });
    xv[eocell[i]] = (b.rhs[s * Ce + i] - o) / b.dS[s * Ce + i];
  });
  for_half(no, [&](int m) { xv[eocell[ne + m]] = xw[ne + m]; });
}

// ============================================================== PCG (Jacobi) for the symmetric p matrix
// scal: 0 rz, 1 rz_prev, 2 alpha, 4 res0, 5 res, 6 active, 7 iters
struct CV { double *dS, *rhs, *r, *z, *pa, *pb, *q, *xw; };

template <int WT, bool FF = false>
__global__ void __launch_bounds__(TPB) k_cg_init(long C, int W, ColView col,
                                                 const double* __restrict__ val, CV v, double* partial,
                                                 FaceOp<double> fo = {}) {
  __shared__ int s_ct[CT_MAX];
  if (!FF) col.stage(s_ct);
  double acc[2] = {0.0, 0.0};
  for (int c = xcd_block() * blockDim.x + threadIdx.x; c < C; c += gridDim.x * blockDim.x) {
    double ax;
    if constexpr (FF) {
      ax = v.dS[c] * v.xw[c];
      face_row(fo, c, [&](int j, double a) { ax += a * v.xw[j]; });
    } else {
      ax = ell_mv<WT>(W, C, col, s_ct, val, v.dS[c], v.xw, c);
    }
    const double rr = v.rhs[c] - ax;
    const double zz = rr / v.dS[c];
    v.r[c] = rr; v.z[c] = zz; v.pa[c] = 0.0; v.pb[c] = 0.0;
    acc[0] += rr * zz; acc[1] += rr * rr;
  }
  block_partials<2>(acc, partial, 0);
}

// prologue: rz, res, convergence, beta; p_new = z + beta p_old (own and, on the fly, neighbours);
// q = A p_new; partial p_new.q
template <int WT, bool FF = false>
__global__ void __launch_bounds__(TPB) k_cg_spmv(long C, int W, ColView col,
                                                 const double* __restrict__ val, int it, int max_iter, double tol,
                                                 double abs_tol, Red red_rz, Red red_rr, double* scal, CV v,
                                                 const double* __restrict__ pold, double* __restrict__ pnew,
                                                 double* partial, RowSet rs, FaceOp<double> fo = {}) {
  if (it > 0 && scal[6] == 0.0) return;   // stopped earlier
  double a[1], b[1];
  red_sum<1>(red_rz, 0, a);
  red_sum<1>(red_rr, 0, b);
  const double rz = a[0], res = sqrt(b[0]);
  const double res0 = it == 0 ? res : scal[4];
  const double rzp = scal[1];
  const bool stop = res <= tol * res0 || res <= abs_tol || it >= max_iter || (it > 0 && rzp == 0.0);
  if (leader() && rs.part != 2) {
    if (it == 0) scal[4] = res;
    if (it == 0 || scal[6] != 0.0) { scal[5] = res; scal[7] = it; }
    scal[6] = stop ? 0.0 : 1.0;
    scal[0] = rz;
  }
  if (stop) return;
  const double beta = it == 0 ? 0.0 : rz / rzp;
  const double* z = v.z;
  const int Wr = WT > 0 ? WT : W;
  __shared__ int s_ct[CT_MAX];
  if (!FF) col.stage(s_ct);
  double acc[1] = {0.0};
  for_rows(C, rs, [&](int c) {
    const double pc = z[c] + beta * pold[c];
    pnew[c] = pc;
    double y = v.dS[c] * pc;
    if constexpr (FF) {
      face_row(fo, c, [&](int j, double a) { y += a * (z[j] + beta * pold[j]); });
    } else {
      const int rb = col.row(c);
#pragma unroll
      for (int k = 0; k < Wr; ++k) {
        const int j = col.get(s_ct, rb, C, k, c);
        y += val[k * C + c] * (z[j] + beta * pold[j]);
      }
    }
    v.q[c] = y;
    acc[0] += pc * y;
  });
  block_partials<1>(acc, partial, 0, rs);
}

// prologue: alpha = rz / (p.q); x += alpha p; r -= alpha q; partials (r.z, r.r); with the Jacobi
// preconditioner also z = r / dS (AMG computes z separately and writes r.z itself)
template <bool JAC>
__global__ void __launch_bounds__(TPB) k_cg_x(long C, Red red, double* scal, double* __restrict__ x, CV v,
                                              const double* __restrict__ pnew, double* partial) {
  if (scal[6] == 0.0) return;
  double pv[1];
  red_sum<1>(red, 0, pv);
  const double rz = scal[0];
  const double alpha = pv[0] != 0.0 ? rz / pv[0] : 0.0;
  if (leader()) { scal[2] = alpha; scal[1] = rz; }
  double acc[2] = {0.0, 0.0};
  for (int c = xcd_block() * blockDim.x + threadIdx.x; c < C; c += gridDim.x * blockDim.x) {
    x[c] = x[c] + alpha * pnew[c];
    const double rr = v.r[c] - alpha * v.q[c];
    v.r[c] = rr;
    if (JAC) {
      const double zz = rr / v.dS[c];
      v.z[c] = zz;
      acc[0] += rr * zz;
    }
    acc[1] += rr * rr;
  }
  block_partials<2>(acc, partial, 0);
}

// ---- several ranks: single-reduction PCG (Chronopoulos & Gear 1989). Every dot product of an iteration --
// gamma = r.z, delta = w.z with w = A z, and ||r||^2 -- goes out in ONE all-gather, where the standard
// recurrence needs two (p.q before alpha, then r.z and r.r after the preconditioner): with p = z + beta p and
// s = w + beta s (= A p, by recurrence), alpha = gamma / (delta - beta gamma / alpha_prev). The SpMV is applied
// to z, so the halo carries z alone (the standard form exchanges z and p_old). Vectors: p in pa, s in pb, w in q.
// scal: 0 gamma, 2 alpha, 4 res0, 5 res, 6 active, 7 iters (as the standard form); 10/11 and 12/13 gamma and alpha
// of even / odd iterations (read by the next iteration's update).

// w = A z over the row set; partial z.w
template <int WT>
__global__ void __launch_bounds__(TPB) k_cgcg_w(long C, int W_, ColView col, const double* __restrict__ val,
                                                const double* scal, int it, CV v, double* partial, RowSet rs) {
  if (it > 0 && scal[6] == 0.0) return;   // stopped (the update kernel of this iteration decided it)
  const int W = WT > 0 ? WT : W_;
  __shared__ int s_ct[CT_MAX];
  col.stage(s_ct);
  double acc[1] = {0.0};
  for_rows(C, rs, [&](int c) {
    const double y = ell_mv<WT>(W, C, col, s_ct, val, v.dS[c], v.z, c);
    v.q[c] = y;
    acc[0] += v.z[c] * y;
  });
  block_partials<1>(acc, partial, 0, rs);
}

// this rank's (||r||^2, r.z, z.w) from the three kernels' block partials, for the one all-gather
__global__ void __launch_bounds__(TPB) k_cgcg_local(Red rr, Red rz, Red zw, const double* scal, int it, double* out) {
  if (it > 0 && scal[6] == 0.0) return;
  double a[1], b[1], c[1];
  red_sum<1>(rr, 0, a);
  red_sum<1>(rz, 0, b);
  red_sum<1>(zw, 0, c);
  if (threadIdx.x == 0) { out[0] = a[0]; out[1] = b[0]; out[2] = c[0]; }
}

// prologue: the gathered (||r||^2, gamma, delta) -> stop test (k_cg_spmv's), beta, alpha; body: p = z + beta p,
// s = w + beta s, x += alpha p, r -= alpha s; partials (r.z [Jacobi: z = r / dS here], r.r)
template <bool JAC>
__global__ void __launch_bounds__(TPB) k_cgcg_update(long C, int it, int max_iter, double tol, double abs_tol, Red red,
                                                     double* scal, double* __restrict__ x, CV v, double* partial) {
  if (it > 0 && scal[6] == 0.0) return;
  double o[3];
  {
    double t[1];
    red_sum<1>(red, 0, t); o[0] = t[0];
    Red r1 = red; r1.p += 1; red_sum<1>(r1, 0, t); o[1] = t[0];
    Red r2 = red; r2.p += 2; red_sum<1>(r2, 0, t); o[2] = t[0];
  }
  const double res = sqrt(o[0]), gamma = o[1], delta = o[2];
  const double res0 = it == 0 ? res : scal[4];
  // gamma and alpha of the previous iteration: slots 10/11 or 12/13 by iteration parity, so no block reads a slot
  // the leader of this launch writes
  const double gp = it == 0 ? 0.0 : scal[10 + 2 * ((it - 1) & 1)], ap = it == 0 ? 0.0 : scal[11 + 2 * ((it - 1) & 1)];
  const bool stop = res <= tol * res0 || res <= abs_tol || it >= max_iter || (it > 0 && (gp == 0.0 || ap == 0.0));
  const double beta = it == 0 ? 0.0 : gamma / gp;
  const double den = it == 0 ? delta : delta - beta * gamma / ap;
  const double alpha = den != 0.0 ? gamma / den : 0.0;
  if (leader()) {
    if (it == 0) scal[4] = res;
    scal[5] = res; scal[7] = it;
    scal[6] = stop ? 0.0 : 1.0;
    scal[0] = gamma; scal[2] = alpha;
    scal[10 + 2 * (it & 1)] = gamma; scal[11 + 2 * (it & 1)] = alpha;
  }
  if (stop) return;
  double acc[2] = {0.0, 0.0};
  for (int c = xcd_block() * blockDim.x + threadIdx.x; c < C; c += gridDim.x * blockDim.x) {
    const double pc = v.z[c] + beta * (it == 0 ? 0.0 : v.pa[c]);
    const double sc = v.q[c] + beta * (it == 0 ? 0.0 : v.pb[c]);
    v.pa[c] = pc; v.pb[c] = sc;
    x[c] = x[c] + alpha * pc;
    const double rr = v.r[c] - alpha * sc;
    v.r[c] = rr;
    if (JAC) {
      const double zz = rr / v.dS[c];
      v.z[c] = zz;
      acc[0] += rr * zz;
    }
    acc[1] += rr * rr;
  }
  block_partials<2>(acc, partial, 0);
}

// k_cg_x<false> fused with the AMG's level-0 first sweep (one rank): the updated residual r (written to
// rnew, the dead z buffer; the host then swaps the r and z roles) is also the
// V-cycle's right-hand side, so the same pass forms x0 = omega r / D and res = r - A x0 in the V-cycle's
// precision T; a neighbour's r_j is re-formed as r_j - alpha q_j (the expression the update stores), so
// x0 and res are bitwise those of k_smooth_res on the stored r. Partials (0, r.r) as k_cg_x<false>.
template <int WT, class T, bool FF = false>
__global__ void __launch_bounds__(TPB) k_cg_x_smooth(long C, int W_, ColView col, Red red,
                                                     double* scal, double* __restrict__ x, CV v,
                                                     const double* __restrict__ pnew, double* __restrict__ rnew,
                                                     double* partial, const T* __restrict__ val0,
                                                     const T* __restrict__ D0, T omega, T* __restrict__ x0,
                                                     T* __restrict__ res0, FaceOp<T> fo = {}) {
  if (scal[6] == 0.0) return;
  double pv[1];
  red_sum<1>(red, 0, pv);
  const double rz = scal[0];
  const double alpha = pv[0] != 0.0 ? rz / pv[0] : 0.0;
  if (leader()) { scal[2] = alpha; scal[1] = rz; }
  const int W = WT > 0 ? WT : W_;
  __shared__ int s_ct[CT_MAX];
  if (!FF) col.stage(s_ct);
  double acc[2] = {0.0, 0.0};
  for (int c = xcd_block() * blockDim.x + threadIdx.x; c < C; c += gridDim.x * blockDim.x) {
    x[c] = x[c] + alpha * pnew[c];
    const double rr = v.r[c] - alpha * v.q[c];
    rnew[c] = rr;   // not in place: neighbours read the old r
    acc[1] += rr * rr;
    const T bc = (T)rr;
    const T xc = omega * bc / D0[c];
    T y = D0[c] * xc;
    if constexpr (FF) {
      face_row(fo, c, [&](int j, T a) {
        if (j < C) y += a * (omega * (T)(v.r[j] - alpha * v.q[j]) / D0[j]);
      });
    } else {
      const int rb = col.row(c);
#pragma unroll
      for (int k = 0; k < W; ++k) {
        const int j = col.get(s_ct, rb, C, k, c);
        if (j < C) y += val0[(long)k * C + c] * (omega * (T)(v.r[j] - alpha * v.q[j]) / D0[j]);
      }
    }
    x0[c] = xc;
    res0[c] = bc - y;
  }
  block_partials<2>(acc, partial, 0);
}

// ============================================================== small systems: one workgroup per solve
// A mesh of a few thousand cells (the 1D flame: 880) runs every iteration kernel at its launch floor
// (≈ 4 µs each, ~500 per step). With one rank and C <= SMALL_C each system's whole solve runs in ONE
// 1024-thread workgroup: the same formulas and stopping tests as the batched kernels above, phases
// separated by workgroup barriers, dot products reduced in fixed order inside the workgroup (so the
// sums are grouped differently from the multi-block reductions: agreement to rounding, not bitwise).
// Vectors stay in global memory (L2-resident at these sizes); all waves of a workgroup share one CU,
// whose L1 the barrier's workgroup-scope fence keeps coherent.
constexpr int SMALL_C = 4096, STPB = 1024, SNW = STPB / 64;

template <int NV> __device__ __forceinline__ void wg_sum(double (&v)[NV]) {
  __shared__ double sh[SNW][NV];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) { const double t = wave_sum(v[k]); if (lane == 0) sh[wid][k] = t; }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    double a = 0.0;
    for (int w = 0; w < SNW; ++w) a += sh[w][k];
    v[k] = a;
  }
  __syncthreads();
}

template <int WT>
__global__ void __launch_bounds__(STPB) k_bcg_small(long C, long Ce, int W_, const int* __restrict__ col,
                                                    const double* __restrict__ val, int max_iter, double tol,
                                                    double abs_tol, double* scal, BV b, Sys q,
                                                    const int* __restrict__ sys_map) {
  const int s = blockIdx.x;
  const int W = WT > 0 ? WT : W_;
  double* st = scal + s * NSCAL;
  const double* vs = val + (long)(b.vshared ? 0 : s) * W * C;
  double *r = b.r + s * Ce, *r0 = b.r0 + s * Ce, *p = b.p + s * Ce, *v = b.v + s * Ce, *t = b.t + s * Ce;
  const double* dS = b.dS + s * Ce;
  double* xv = q.x + (sys_map ? sys_map[s] : s) * q.xstride;
  // r = D^-1 (b - A x); r0 = p = r (k_bcg_init)
  double a2[2] = {0.0, 0.0};
  for (int c = threadIdx.x; c < C; c += STPB) {
    const double d = dS[c];
    const double res = b.rhs[s * Ce + c] - ell_mv<WT>(W, C, ColView{col, nullptr, nullptr, W}, nullptr, vs, d, b.xw + s * Ce, c);
    const double rr = res / d;
    r[c] = rr; r0[c] = rr; p[c] = rr;
    a2[0] += res * res;
    a2[1] += rr * rr;
  }
  wg_sum<2>(a2);
  const double res0 = sqrt(a2[0]);
  double n2 = a2[0], rho = a2[1], omega = 1.0;
  int it = 0;
  for (;; ++it) {
    const double res = sqrt(n2);
    const bool stop = res <= tol * res0 || res <= abs_tol || it >= max_iter || (it > 0 && (rho == 0.0 || omega == 0.0));
    if (threadIdx.x == 0) { st[4] = res0; st[0] = rho; st[5] = res; st[7] = it; st[6] = stop ? 0.0 : 1.0; }
    if (stop) break;
    // v = D^-1 A p; r0.v
    double a1[1] = {0.0};
    for (int c = threadIdx.x; c < C; c += STPB) {
      const double y = scaled_mv<WT>(W, C, ColView{col, nullptr, nullptr, W}, nullptr, vs, dS[c], p, c);
      v[c] = y;
      a1[0] += r0[c] * y;
    }
    wg_sum<1>(a1);
    const double alpha = a1[0] != 0.0 ? rho / a1[0] : 0.0;
    // t = D^-1 A s, s = r - alpha v formed on the fly; (t.s, t.t, r0.t, r0.s)
    double a4[4] = {0.0, 0.0, 0.0, 0.0};
    for (int c = threadIdx.x; c < C; c += STPB) {
      const double sc = r[c] - alpha * v[c];
      double o = 0.0;
#pragma unroll
      for (int k = 0; k < W; ++k) {
        const int j = col[k * C + c];
        o += vs[k * C + c] * (r[j] - alpha * v[j]);
      }
      const double y = sc + o / dS[c];
      t[c] = y;
      const double rz = r0[c];
      a4[0] += y * sc; a4[1] += y * y; a4[2] += rz * y; a4[3] += rz * sc;
    }
    wg_sum<4>(a4);
    omega = a4[1] != 0.0 ? a4[0] / a4[1] : 0.0;
    const double rho_new = a4[3] - omega * a4[2];
    const double beta = (rho != 0.0 && omega != 0.0) ? (rho_new / rho) * (alpha / omega) : 0.0;
    // x += alpha p + omega s; r = s - omega t; p = r + beta (p - omega v); ||D r||^2
    a1[0] = 0.0;
    for (int c = threadIdx.x; c < C; c += STPB) {
      const double pv = p[c], vv = v[c];
      const double sv = r[c] - alpha * vv;
      xv[c] = xv[c] + alpha * pv + omega * sv;
      const double rr = sv - omega * t[c];
      r[c] = rr;
      p[c] = rr + beta * (pv - omega * vv);
      const double tr = dS[c] * rr;
      a1[0] += tr * tr;
    }
    wg_sum<1>(a1);
    n2 = a1[0];
    rho = rho_new;
    if (threadIdx.x == 0) { st[3] = omega; st[1] = st[0]; st[8] = rho_new; }
  }
  if (threadIdx.x == 0) st[6] = 0.0;
}

// the AMG V-cycle of amg.hip (k_smooth_res, k_restrict, k_coarsest, k_prolong_smooth, same arithmetic
// per cell) inside one workgroup: z = M^-1 r, returns r.z (every thread)
template <class T>
__device__ double vcycle_wg(const AmgView<T>& a, const double* __restrict__ r0, double* __restrict__ z) {
  const int L = a.L;
  const T om = a.omega, sc = a.sc;
  if (L == 1) {   // a single level (double): Jacobi sweeps from zero straight into z (k_coarsest)
    const int n = a.n[0], W = a.W[0];
    const int* col = a.col[0];
    const T *val = a.val[0], *D = a.D[0];
    T* xa = a.x[0];
    T* xb = a.r[0];
    for (int c = threadIdx.x; c < n; c += STPB) xa[c] = om * (T)r0[c] / D[c];
    __syncthreads();
    for (int sw = 1; sw < a.sweeps; ++sw) {
      for (int c = threadIdx.x; c < n; c += STPB) {
        T y = D[c] * xa[c];
        for (int k = 0; k < W; ++k) { const int j = col[k * n + c]; if (j < n) y += val[k * n + c] * xa[j]; }
        xb[c] = xa[c] + om * ((T)r0[c] - y) / D[c];
      }
      __syncthreads();
      T* tt = xa; xa = xb; xb = tt;
    }
    double acc[1] = {0.0};
    for (int c = threadIdx.x; c < n; c += STPB) { z[c] = (double)xa[c]; acc[0] += r0[c] * (double)xa[c]; }
    wg_sum<1>(acc);
    return acc[0];
  }
  // down: one sweep from zero + residual, restriction
  for (int l = 0; l + 1 < L; ++l) {
    const int n = a.n[l], W = a.W[l];
    const int* col = a.col[l];
    const T *val = a.val[l], *D = a.D[l];
    for (int c = threadIdx.x; c < n; c += STPB) {
      const T bc = l == 0 ? (T)r0[c] : a.b[l][c];
      const T xc = om * bc / D[c];
      T y = D[c] * xc;
      for (int k = 0; k < W; ++k) {
        const int j = col[(long)k * n + c];
        if (j < n) y += val[(long)k * n + c] * (om * (l == 0 ? (T)r0[j] : a.b[l][j]) / D[j]);
      }
      a.x[l][c] = xc;
      a.r[l][c] = bc - y;
    }
    __syncthreads();
    const int nc = a.n[l + 1];
    for (int I = threadIdx.x; I < nc; I += STPB) {
      T sm = 0;
      for (int e = a.mstart[l][I]; e < a.mstart[l][I + 1]; ++e) sm += a.r[l][a.members[l][e]];
      a.b[l + 1][I] = sm;
    }
    __syncthreads();
  }
  {   // coarsest: weighted-Jacobi sweeps from zero (ping-pong through x / r of that level)
    const int l = L - 1, n = a.n[l], W = a.W[l];
    const int* col = a.col[l];
    const T *val = a.val[l], *D = a.D[l], *bb = a.b[l];
    T* xa = a.x[l];
    T* xb = a.r[l];
    for (int c = threadIdx.x; c < n; c += STPB) xa[c] = om * bb[c] / D[c];
    __syncthreads();
    for (int sw = 1; sw < a.sweeps; ++sw) {
      for (int c = threadIdx.x; c < n; c += STPB) {
        T y = D[c] * xa[c];
        for (int k = 0; k < W; ++k) { const int j = col[k * n + c]; if (j < n) y += val[k * n + c] * xa[j]; }
        xb[c] = xa[c] + om * (bb[c] - y) / D[c];
      }
      __syncthreads();
      T* tt = xa; xa = xb; xb = tt;
    }
    if (xa != a.x[l]) {   // the result in x[l]
      for (int c = threadIdx.x; c < n; c += STPB) a.x[l][c] = xa[c];
      __syncthreads();
    }
  }
  // up: prolongate the scaled coarse correction + one sweep; levels >= 1 into xo, level 0 into z
  for (int l = L - 2; l >= 1; --l) {
    const int n = a.n[l], W = a.W[l];
    const int* col = a.col[l];
    const int* agg = a.agg[l];
    const T *val = a.val[l], *D = a.D[l], *bb = a.b[l], *x = a.x[l];
    const T* xc = l + 1 == L - 1 ? a.x[l + 1] : a.xo[l + 1];
    for (int c = threadIdx.x; c < n; c += STPB) {
      const T yc = x[c] + sc * xc[agg[c]];
      T ay = D[c] * yc;
      for (int k = 0; k < W; ++k) {
        const int j = col[(long)k * n + c];
        if (j < n) ay += val[(long)k * n + c] * (x[j] + sc * xc[agg[j]]);
      }
      a.xo[l][c] = yc + om * (bb[c] - ay) / D[c];
    }
    __syncthreads();
  }
  const int n = a.n[0], W = a.W[0];
  const int* col = a.col[0];
  const int* agg = a.agg[0];
  const T *val = a.val[0], *D = a.D[0], *x = a.x[0];
  const T* xc = L == 2 ? a.x[1] : a.xo[1];
  double acc[1] = {0.0};
  for (int c = threadIdx.x; c < n; c += STPB) {
    const T yc = x[c] + sc * xc[agg[c]];
    T ay = D[c] * yc;
    for (int k = 0; k < W; ++k) {
      const int j = col[(long)k * n + c];
      if (j < n) ay += val[(long)k * n + c] * (x[j] + sc * xc[agg[j]]);
    }
    const double bc = r0[c];
    const double o = (double)(yc + om * ((T)bc - ay) / D[c]);
    z[c] = o;
    acc[0] += bc * o;
  }
  wg_sum<1>(acc);
  return acc[0];
}

// the whole PCG solve (k_cg_init, k_cg_spmv, k_cg_x and the preconditioner) in one workgroup; AMG:
// the V-cycle above, otherwise Jacobi (z = r / dS)
template <int WT, class T, bool AMG>
__global__ void __launch_bounds__(STPB) k_pcg_small(long C, int W_, const int* __restrict__ col,
                                                    const double* __restrict__ val, int max_iter, double tol,
                                                    double abs_tol, double* scal, CV v, double* __restrict__ xsol,
                                                    AmgView<T> a) {
  const int W = WT > 0 ? WT : W_;
  double* p = v.pa;
  double a2[2] = {0.0, 0.0};
  for (int c = threadIdx.x; c < C; c += STPB) {
    const double rr = v.rhs[c] - ell_mv<WT>(W, C, ColView{col, nullptr, nullptr, W}, nullptr, val, v.dS[c], v.xw, c);
    v.r[c] = rr;
    p[c] = 0.0;
    if (!AMG) { const double zz = rr / v.dS[c]; v.z[c] = zz; a2[0] += rr * zz; }
    a2[1] += rr * rr;
  }
  wg_sum<2>(a2);
  double rz = a2[0], rr2 = a2[1];
  if constexpr (AMG) rz = vcycle_wg<T>(a, v.r, v.z);
  const double res0 = sqrt(rr2);
  double rzp = 0.0;
  for (int it = 0;; ++it) {
    const double res = sqrt(rr2);
    const bool stop = res <= tol * res0 || res <= abs_tol || it >= max_iter || (it > 0 && rzp == 0.0);
    if (threadIdx.x == 0) { scal[4] = res0; scal[5] = res; scal[7] = it; scal[6] = stop ? 0.0 : 1.0; scal[0] = rz; }
    if (stop) break;
    const double beta = it == 0 ? 0.0 : rz / rzp;
    for (int c = threadIdx.x; c < C; c += STPB) p[c] = v.z[c] + beta * p[c];
    __syncthreads();
    double a1[1] = {0.0};
    for (int c = threadIdx.x; c < C; c += STPB) {
      double y = v.dS[c] * p[c];
#pragma unroll
      for (int k = 0; k < W; ++k) y += val[k * C + c] * p[col[k * C + c]];
      v.q[c] = y;
      a1[0] += p[c] * y;
    }
    wg_sum<1>(a1);
    const double alpha = a1[0] != 0.0 ? rz / a1[0] : 0.0;
    a2[0] = 0.0; a2[1] = 0.0;
    for (int c = threadIdx.x; c < C; c += STPB) {
      xsol[c] = xsol[c] + alpha * p[c];
      const double rr = v.r[c] - alpha * v.q[c];
      v.r[c] = rr;
      if (!AMG) { const double zz = rr / v.dS[c]; v.z[c] = zz; a2[0] += rr * zz; }
      a2[1] += rr * rr;
    }
    wg_sum<2>(a2);
    rzp = rz;
    rr2 = a2[1];
    if constexpr (AMG) rz = vcycle_wg<T>(a, v.r, v.z);
    else rz = a2[0];
    if (threadIdx.x == 0) { scal[2] = alpha; scal[1] = rzp; }
  }
  if (threadIdx.x == 0) scal[6] = 0.0;
}

// ------------------------------------------------------------------ host side
struct Launch {
  Ctx& x;
  int nblk, nsys;
  // make the partials of the last kernel readable by the next (slot: independent buffers for
  // reductions that are alive at the same time)
  Red after(double* partial, int NV, int slot = 0, int np = 0) {
    if (np == 0) np = nblk;
    if (x.nranks == 1) return Red{partial, np, NV, (long)np * NV};
    const size_t per = (size_t)nsys * 4;   // up to 4 values per system per slot
    if (x.sws().red_local.n < 2 * per) x.sws().red_local.alloc(2 * per);
    if (x.sws().red_all.n < 2 * per * x.nranks) x.sws().red_all.alloc(2 * per * x.nranks);
    double* loc = x.sws().red_local.p + slot * per;
    double* all = x.sws().red_all.p + slot * per * x.nranks;
    if (NV == 1) hipLaunchKernelGGL(k_red_local<1>, dim3(nsys), dim3(TPB), 0, x.stream, partial, np, loc);
    else if (NV == 2) hipLaunchKernelGGL(k_red_local<2>, dim3(nsys), dim3(TPB), 0, x.stream, partial, np, loc);
    else if (NV == 3) hipLaunchKernelGGL(k_red_local<3>, dim3(nsys), dim3(TPB), 0, x.stream, partial, np, loc);
    else hipLaunchKernelGGL(k_red_local<4>, dim3(nsys), dim3(TPB), 0, x.stream, partial, np, loc);
    DFMI_HIP(hipGetLastError());
    halo_allgather(x, loc, all, (long)nsys * NV);
    return Red{all, x.nranks, (long)nsys * NV, NV};
  }
};

template <class F> void dispatch_W(int W, F&& f) {
  switch (W) {
    case 4: f(std::integral_constant<int, 4>()); break;
    case 5: f(std::integral_constant<int, 5>()); break;
    case 6: f(std::integral_constant<int, 6>()); break;
    default: f(std::integral_constant<int, 0>()); break;
  }
}

void halo_vecs(Ctx& x, std::initializer_list<double*> vecs, int nsys, long Ce, bool split = false, int colour = -1) {
  if (!halo_active(x)) return;
  std::vector<HaloItem> it;
  for (double* v : vecs) it.push_back({v, v, nsys, Ce, Ce, false, split, colour});
  halo_update(x, it.data(), (int)it.size());
}

// An SpMV-type launch that reads the halo entries of `vecs`: with overlap, the interior rows run while
// the exchange is in flight and the boundary rows after it (partials in two halves, np = 2 nblk);
// otherwise exchange, then all rows. launch(RowSet) enqueues the kernel; returns the partial count.
template <class F>
int spmv_with_halo(Ctx& x, std::initializer_list<double*> vecs, int nsys, long Ce, int nblk, F&& launch) {
  if (!halo_overlap(x)) {
    halo_vecs(x, vecs, nsys, Ce);
    launch(RowSet{});
    return nblk;
  }
  std::vector<HaloItem> it;
  for (double* v : vecs) it.push_back({v, v, nsys, Ce, Ce, false});
  halo_begin(x, it.data(), (int)it.size());
  launch(RowSet{1, x.ell.bflag.p, x.ell.brow.p, x.ell.nb});
  halo_end(x);
  launch(RowSet{2, x.ell.bflag.p, x.ell.brow.p, x.ell.nb});
  return 2 * nblk;
}

// one rank, no halo, a few thousand cells: each solve in one workgroup launch (solver.small = 0: off)
bool small_solve(const Ctx& x) {
  if (x.nranks != 1 || halo_active(x) || x.C > SMALL_C || x.C == 0) return false;
  return x.on("solver.small");
}

// Convergence polling without draining the stream: after an iteration a one-wave kernel posts the solve's state
// (every system stopped?, iterations) into host-coherent pinned memory, and the host reads the record of an
// EARLIER check -- the GPU is already running the next iteration(s) by then (systems that stopped turn every
// kernel into an early return), so the queue never empties inside a solve. The decision is a pure function of
// the globally reduced scalars, identical on every rank.
// Cadence (round 5): the iterations the previous solve of the same equation needed (`expect`, 0 = none yet)
// place the checks. Before expect - 1 a record every 4 iterations (a solve that converges early costs a few
// early-return launches more); from there a record after EVERY iteration, each check reading the one an
// iteration back, so a converged solve is stopped one iteration after the one that set its flag. The round-4
// cadence (a snapshot every 2 iterations, read 2 later) ran 3-4 iterations of early-return launches after every
// solve (~4.7 us each: 0.3 ms per p-solve, ~1.2 ms per step, profiles/r05_timeline_poll.json), and each
// snapshot was a device-to-host copy plus an event (~10 us of the stream); the posted record is one small launch.
__global__ void k_poll_post(const double* __restrict__ scal, int nsys, PollRec* rec, long long seq) {
  poll_post(scal, nsys, rec, seq);
}

struct Poller {
  Ctx& x;
  const double* scal;
  int nsys;
  long long pending = 0;   // the record a check waits for (0: none)
  int expect;
  std::string key;
  Poller(Ctx& c, const double* s, int n, const std::string& k) : x(c), scal(s), nsys(n), key(k) {
    x.sws().poll.ensure();
    auto f = x.solve_expect.find(key);
    expect = f == x.solve_expect.end() ? 0 : f->second;
  }
  // wait (spinning) until record `seq` or a later one is posted; a stream that drained without posting it
  // (a failed launch) is an error rather than a hang
  const PollRec& wait(long long seq) {
    const PollRec* r = x.sws().poll.h + (seq & 1);
    for (long spins = 0;; ++spins) {
      if (__atomic_load_n(&r->seq, __ATOMIC_ACQUIRE) >= seq) return *r;
      if ((spins & 0xfff) == 0xfff) {
        const hipError_t q = hipStreamQuery(x.stream);
        if (q != hipErrorNotReady && __atomic_load_n(&r->seq, __ATOMIC_ACQUIRE) < seq) {
          DFMI_HIP(q);
          throw Error("solver poll: the stream drained without posting its convergence record");
        }
      }
    }
  }
  long long next = 0;      // the record the current iteration posts (0: none)
  // before iteration `it`'s (0-based) last kernel is enqueued: the sequence number of the record this iteration
  // posts when the cadence says so, else 0 (a caller may have that kernel post it: k_eo_xp)
  long long plan(int it) {
    const int n = it + 1;
    const bool snap = expect > 0 ? (n >= expect - 1 || n % 4 == 0) : (n % 2 == 0);
    next = snap ? ++x.sws().poll_seq : 0;
    return next;
  }
  // after the iteration was enqueued (with its record, if plan() asked for one): true when an earlier record
  // shows every system stopped (its iteration count becomes the next solve's `expect`)
  bool check() {
    if (!next) return false;
    if (x.nranks > 1) {
      // several ranks: wait for the record just posted (lag 0). An iteration enqueued after convergence costs
      // its halo exchanges and all-gathers in full -- transport calls are not skipped by the device's flags
      // (4 halos + 2 all-gathers of an even-odd BiCGStab iteration, 3 + 1 of the PCG) -- while the bubble of
      // waiting here is one host reaction
      const PollRec& r = wait(next);
      pending = 0;
      if (r.stopped) {
        x.solve_expect[key] = r.iters;
        return true;
      }
      return false;
    }
    bool done = false;
    if (pending > 0) {
      const PollRec& r = wait(pending);
      if (r.stopped) {
        done = true;
        x.solve_expect[key] = r.iters;
      }
    }
    pending = next;
    return done;
  }
  // the same with the record posted by its own one-wave launch
  bool after(int it) {
    const long long seq = plan(it);
    if (!seq) return false;
    hipLaunchKernelGGL(k_poll_post, dim3(1), dim3(64), 0, x.stream, scal, nsys, x.sws().poll.d, seq);
    DFMI_HIP(hipGetLastError());
    return check();
  }
};

int work_slot(const std::string& eqn) {
  if (eqn == "U") return 0;
  if (eqn == "Y") return 1;
  if (eqn == "E") return 2;
  if (eqn == "p") return 3;
  throw Error("dfmi: unknown equation '" + eqn + "'");
}

// the solve's scalars stored straight into the mapped host snapshot (vector stores; one launch instead of a launch and
// a copy), and its system-iterations summed into the equation's work counter
__global__ void k_accum_iters(const double* scal, int nsys, double* acc, double* snap) {
  for (int i = threadIdx.x; i < nsys * NSCAL; i += blockDim.x) snap[i] = scal[i];
  if (threadIdx.x != 0) return;
  double a = 0.0;
  for (int s = 0; s < nsys; ++s) a += scal[s * NSCAL + 7];
  *acc += a;
}

// final state of the solve, recorded for dfmi_solver_stats without waiting (it synchronises before reading);
// iterations summed into the equation's work counter on the device
void record_stats(Ctx& x, const char* eqn, const double* scal, int nsys) {
  if (x.work.n == 0) { x.work.alloc(4); x.work.zero(x.stream); }
  auto& sn = x.stat_snap[eqn];
  sn.h.ensure_mapped((size_t)nsys * NSCAL);
  sn.nsys = nsys;
  hipLaunchKernelGGL(k_accum_iters, dim3(1), dim3(64), 0, x.stream, scal, nsys, x.work.p + work_slot(eqn), sn.h.d);
}

}  // namespace

void build_ell(Ctx& x) {
  const int C = x.C;
  std::vector<int> own = x.h_own, nei = x.h_nei;
  std::vector<std::vector<std::pair<int, int>>> ent(C);   // (col, src)
  std::vector<std::vector<int>> nbrf(C);
  for (int f = 0; f < x.F; ++f) nbrf[nei[f]].push_back(f);
  // coefficient sources by face STORAGE index (lower/upper live in the owner-slot layout)
  for (int c = 0; c < C; ++c) for (int f : nbrf[c]) ent[c].push_back({own[f], 2 * x.h_fst[f]});
  for (int f = 0; f < x.F; ++f) ent[own[f]].push_back({nei[f], 2 * x.h_fst[f] + 1});
  // owned faces were appended in ascending face order after the neighbour faces: matches each_face
  std::vector<int> partner(x.B, -1);
  for (int p = 0; p < x.P; ++p) {
    if (x.pkind[p] != 1) continue;
    const int q = x.cyc_nbr[p];
    for (int i = 0; i < x.psize[p]; ++i) partner[x.poff[p] + i] = x.h_bfc[x.poff[q] + i];
  }
  for (int p = 0; p < x.P; ++p) {   // coupled primary slots in slot order (= cbSlot order per cell)
    if (x.pkind[p] == 0) continue;
    for (int i = 0; i < x.psize[p]; ++i) {
      const int b = x.poff[p] + i;
      const int c = x.h_bfc[b];
      int colv;
      if (x.pkind[p] == 1) colv = partner[b];
      else {
        DFMI_CHECK(halo_active(x) && b < (int)x.h_hidx.size() && x.h_hidx[b] >= 0,
                   "processor patches need dfmi_set_comm_info before the first solve");
        colv = C + x.h_hidx[b];
      }
      ent[c].push_back({colv, -(b + 1)});
    }
  }
  int W = 0;
  for (auto& e : ent) W = std::max(W, (int)e.size());
  W = std::max(W, 1);
  std::vector<int> col((size_t)W * C), src((size_t)W * C);
  for (int c = 0; c < C; ++c)
    for (int k = 0; k < W; ++k) {
      const bool have = k < (int)ent[c].size();
      col[(size_t)k * C + c] = have ? ent[c][k].first : c;
      src[(size_t)k * C + c] = have ? ent[c][k].second : PAD;
    }
  x.ell.W = W;
  x.ell.col.upload(col, x.stream);
  x.ell.src.upload(src, x.stream);
  std::vector<int8_t> bflag(C, 0);
  std::vector<int> brow;
  for (int c = 0; c < C; ++c) {
    for (auto& e : ent[c]) if (e.first >= C) bflag[c] = 1;
    if (bflag[c]) brow.push_back(c);
  }
  x.ell.nb = (int)brow.size();
  if (brow.empty()) brow.push_back(0);
  x.ell.bflag.upload(bflag, x.stream);
  {   // coupled slots per cell (the ELL's slot entries, ascending slot index) and their columns (FaceOp)
    std::vector<int> cs(C + 1, 0), sl, scol(std::max(x.B, 1), 0);
    for (int c = 0; c < C; ++c) {
      for (auto& e : ent[c])
        if (e.second < 0 && e.second != PAD) { sl.push_back(-e.second - 1); scol[-e.second - 1] = e.first; }
      cs[c + 1] = (int)sl.size();
    }
    if (sl.empty()) sl.push_back(0);
    x.ell.csStart.upload(cs, x.stream);
    x.ell.csSlot.upload(sl, x.stream);
    x.ell.scol.upload(scol, x.stream);
  }
  x.ell.brow.upload(brow, x.stream);
  // hex box in blockMesh order (MeshView::hx, each_face<-1>): nx and nx ny from the face offsets, then every
  // cell's face entries checked against the computed walk (same faces, storage indices, order)
  x.hex[0] = x.hex[1] = x.hex[2] = 0;
  if (x.fslot && x.F > 0) {
    int nx = 0, nxy = 0;
    bool ok = true;
    for (int f = 0; f < x.F && ok; ++f) {
      const int d = x.h_nei[f] - x.h_own[f];
      if (d > 1 && (nx == 0 || d < nx)) nx = d;
      nxy = std::max(nxy, d);
      ok = d > 0;
    }
    if (ok && nx > 1 && nxy > nx && nxy % nx == 0 && C % nxy == 0) {
      const int ny = nxy / nx, nz = C / nxy;
      for (int c = 0; c < C && ok; ++c) {
        const int t = c / nx, i = c - t * nx, k = t / ny, j = t - k * ny;
        const int hxp = i < nx - 1, hyp = j < ny - 1;
        int sf[6], so[6], sw[6], n = 0;
        auto add = [&](int f, int o, int w) { sf[n] = f; so[n] = o; sw[n] = w; ++n; };
        if (k > 0) add((hxp + hyp) * C + c - nxy, c - nxy, 0);
        if (j > 0) add(hxp * C + c - nx, c - nx, 0);
        if (i > 0) add(c - 1, c - 1, 0);
        if (hxp) add(c, c + 1, 1);
        if (hyp) add(hxp * C + c, c + nx, 1);
        if (k < nz - 1) add((hxp + hyp) * C + c, c + nxy, 1);
        int q = 0;
        for (int kk = 0; kk < W && ok; ++kk) {
          const int s = src[(size_t)kk * C + c];
          if (s < 0) continue;   // slot or padding: not part of the face walk
          ok = q < n && (s >> 1) == sf[q] && (s & 1) == sw[q] && col[(size_t)kk * C + c] == so[q];
          ++q;
        }
        ok = ok && q == n;
      }
      if (ok) { x.hex[0] = nx; x.hex[1] = ny; x.hex[2] = nz; }
    }
  }
  // even-odd layout of the BiCGStab rows (k_eo_*): not the one-workgroup small solves, and a coupling graph
  // that 2-colours -- every ELL entry couples the other colour (cyclic partners included; a periodic direction
  // of odd extent does not colour and keeps the Jacobi path). Several ranks: each rank's (connected) local
  // graph is coloured, the colours across every processor face are exchanged, and the ranks' flips are solved
  // from the all-gathered relations so that every processor face couples the two colours too -- the same
  // decision on every rank. solver.even_odd = 0: off
  x.ell.eo = 0;
  x.ell.eo_ncls = 0;
  x.ell.h_eo_pos.clear();
  const bool multi = x.nranks > 1 && x.halo != nullptr;
  if (x.on("solver.even_odd") && !small_solve(x) && (multi || !halo_active(x))) {
    std::vector<int> colr(C, 0), q;
    std::vector<char> seen(C, 0);
    bool bip = C >= 2;
    int ncomp = 0;
    for (int c0 = 0; c0 < C && bip; ++c0) {
      if (seen[c0]) continue;
      ++ncomp;
      seen[c0] = 1;
      colr[c0] = 0;
      q.assign(1, c0);
      for (size_t h = 0; h < q.size() && bip; ++h) {
        const int c = q[h];
        for (int k = 0; k < W; ++k) {
          if (src[(size_t)k * C + c] == PAD) continue;
          const int j = col[(size_t)k * C + c];
          if (j >= C && multi) continue;   // a processor column: checked across ranks below
          if (j < 0 || j >= C || j == c) { bip = false; break; }
          if (!seen[j]) { seen[j] = 1; colr[j] = 1 - colr[c]; q.push_back(j); }
          else if (colr[j] == colr[c]) { bip = false; break; }
        }
      }
    }
    int ne = 0;
    for (int c = 0; c < C; ++c) ne += colr[c] == 0;
    bip = bip && ne > 0 && ne < C;
    if (multi) {
      // colour of the cell across every processor face -> per peer the flip relation f_rank ^ f_peer this rank
      // needs (one value for all its faces with that peer, else 2); all-gathered with a local ok flag
      const int R = x.nranks;
      const long Ce = (long)C + x.H;
      std::vector<double> cd(Ce, 0.0);
      for (int c = 0; c < C; ++c) cd[c] = colr[c];
      DevBuf<double> dcd;
      dcd.upload(cd, x.stream);
      if (halo_active(x)) {
        HaloItem it{dcd.p, dcd.p, 1, Ce, Ce, false};
        halo_update(x, &it, 1);
      }
      DFMI_HIP(hipMemcpyAsync(cd.data(), dcd.p, Ce * sizeof(double), hipMemcpyDeviceToHost, x.stream));
      DFMI_HIP(hipStreamSynchronize(x.stream));
      const std::vector<int> peer = halo_peers_of(x);
      std::vector<double> row(R + 1, -1.0);
      row[R] = (bip && ncomp == 1) ? 1.0 : 0.0;
      for (int c = 0; c < C; ++c)
        for (int k = 0; k < W; ++k) {
          const int j = col[(size_t)k * C + c];
          if (src[(size_t)k * C + c] == PAD || j < C) continue;
          const int pr = peer[j - C];
          const double d = (double)(1 ^ colr[c] ^ (int)cd[j]);
          if (row[pr] < 0) row[pr] = d;
          else if (row[pr] != d) row[pr] = 2.0;
        }
      DevBuf<double> sb, rb;
      sb.upload(row, x.stream);
      rb.alloc((size_t)R * (R + 1));
      halo_allgather(x, sb.p, rb.p, R + 1);
      std::vector<double> all((size_t)R * (R + 1));
      DFMI_HIP(hipMemcpyAsync(all.data(), rb.p, all.size() * sizeof(double), hipMemcpyDeviceToHost, x.stream));
      DFMI_HIP(hipStreamSynchronize(x.stream));
      bool ok = true;
      for (int r = 0; r < R; ++r) ok = ok && all[(size_t)r * (R + 1) + R] == 1.0;
      std::vector<int> f(R, -1);
      for (int r0 = 0; r0 < R && ok; ++r0) {   // flips: BFS over the rank graph, the same on every rank
        if (f[r0] >= 0) continue;
        f[r0] = 0;
        std::vector<int> rq(1, r0);
        for (size_t a = 0; a < rq.size() && ok; ++a) {
          const int r = rq[a];
          for (int qr = 0; qr < R && ok; ++qr) {
            const double d = all[(size_t)r * (R + 1) + qr], d2 = all[(size_t)qr * (R + 1) + r];
            if (d < 0) continue;
            if (d > 1.5 || (d2 >= 0 && d2 != d)) { ok = false; break; }
            const int fq = f[r] ^ (int)d;
            if (f[qr] < 0) { f[qr] = fq; rq.push_back(qr); }
            else if (f[qr] != fq) ok = false;
          }
        }
      }
      bip = ok;
      if (ok && f[x.rank] == 1) {
        for (int c = 0; c < C; ++c) colr[c] ^= 1;
        ne = C - ne;
      }
    }
    if (bip) {
      const int no = C - ne;
      std::vector<int> pos(C), cell(C);
      for (int c = 0, a = 0, o = ne; c < C; ++c) {
        const int r = colr[c] == 0 ? a++ : o++;
        pos[c] = r; cell[r] = c;
      }
      std::vector<int> ecol((size_t)W * C);
      for (int c = 0; c < C; ++c) {
        const int i = pos[c];
        for (int k = 0; k < W; ++k) {
          const int j = col[(size_t)k * C + c];
          int jj;
          if (src[(size_t)k * C + c] == PAD)   // value 0: any row of the other colour (the same offset where possible)
            jj = colr[c] == 0 ? ne + std::min(i, no - 1) : std::min(i - ne, ne - 1);
          else jj = j >= C ? j : pos[j];        // processor columns keep their halo index C + h
          ecol[(size_t)k * C + i] = jj;
        }
      }
      x.ell.eo_pos.upload(pos, x.stream);
      x.ell.eo_cell.upload(cell, x.stream);
      x.ell.eo_col.upload(ecol, x.stream);
      // row classes of the reordered rows (column offsets only: the solver reads no sources; halo columns
      // stay explicit)
      std::map<std::vector<int>, int> ids;
      std::vector<uint8_t> cls(C);
      std::vector<int> key(W);
      bool ok = true;
      for (int i = 0; i < C && ok; ++i) {
        for (int k = 0; k < W; ++k) {
          const int jj = ecol[(size_t)k * C + i];
          key[k] = jj >= C ? CEXPL : jj - i;
        }
        auto it = ids.find(key);
        if (it == ids.end()) {
          if (ids.size() >= 255) { ok = false; break; }
          it = ids.emplace(key, (int)ids.size()).first;
        }
        cls[i] = (uint8_t)it->second;
      }
      if (ok && (long)ids.size() * W <= CT_MAX) {
        std::vector<int> ctab(ids.size() * (size_t)W);
        for (auto& kv : ids)
          for (int k = 0; k < W; ++k) ctab[(size_t)kv.second * W + k] = kv.first[k];
        x.ell.eo_cls.upload(cls, x.stream);
        x.ell.eo_ctab.upload(ctab, x.stream);
        x.ell.eo_ncls = (int)ids.size();
      }
      x.ell.h_eo_pos = pos;
      x.ell.ne = ne;
      x.ell.eo = 1;
      if (multi) halo_set_split(x);
    }
  }
  // row classes: per cell the W (column offset, source code) pairs; coupled slots keep explicit sources
  // (slot ids are not relative to the cell) and processor columns explicit columns
  x.ell.ncls = 0;
  if (x.fslot && x.on("solver.row_classes")) {
    std::map<std::vector<int>, int> ids;
    std::vector<uint8_t> cls(C);
    std::vector<int> key(2 * W);
    bool ok = true;
    for (int c = 0; c < C && ok; ++c) {
      for (int k = 0; k < W; ++k) {
        const int j = col[(size_t)k * C + c], s = src[(size_t)k * C + c];
        int co, sc;
        if (s == PAD) { co = j - c; sc = SCODE_PAD; }
        else if (s < 0) { co = j < C ? j - c : CEXPL; sc = CEXPL; }
        else {
          const int fs = s >> 1, own = s & 1, owner = own ? c : j;
          const int ks = (fs - owner) / C;
          ok = ok && (long)ks * C + owner == fs;
          co = j - c; sc = 2 * ks + own;
        }
        key[k] = co; key[W + k] = sc;
      }
      auto it = ids.find(key);
      if (it == ids.end()) {
        if (ids.size() >= 255) { ok = false; break; }
        it = ids.emplace(key, (int)ids.size()).first;
      }
      cls[c] = (uint8_t)it->second;
    }
    if (ok && C > 0 && (long)ids.size() * W <= CT_MAX) {
      const int n = (int)ids.size();
      std::vector<int> ctab((size_t)n * W), stab((size_t)n * W);
      for (auto& kv : ids)
        for (int k = 0; k < W; ++k) { ctab[(size_t)kv.second * W + k] = kv.first[k]; stab[(size_t)kv.second * W + k] = kv.first[W + k]; }
      x.ell.cls.upload(cls, x.stream);
      x.ell.ctab.upload(ctab, x.stream);
      x.ell.stab.upload(stab, x.stream);
      x.ell.ncls = n;
    }
  }
  DFMI_HIP(hipStreamSynchronize(x.stream));
  x.ell.ready = true;
}


// BiCGStab workspace: BCG_VECS vectors of nsys * (C + H), then the ELL values [nsys][W][C], then partials.
// Assembly kernels that emit the ELL form directly (y_assemble_ell) write into it before the solve.
void bicg_layout(Ctx& x, int nsys, double** val, double** dS, double** rhs) {
  if (!x.ell.ready) build_ell(x);
  const long C = x.C, Ce = (long)x.C + x.H;
  const int W = x.ell.W;
  const int nblk = std::min(blocks_for(C, TPB), MAX_BLOCKS);
  const size_t need = (size_t)BCG_VECS * nsys * Ce + (size_t)nsys * W * C +
                      (size_t)nsys * std::max(nblk, eo_max_blocks()) * 12 + 64;
  if (x.sws().buf.n < need) { x.sws().buf.alloc(need); x.sws().buf.zero(x.stream); }   // no stale NaN under a 0 coefficient
  const long N = nsys * Ce;
  *dS = x.sws().buf.p;
  *rhs = x.sws().buf.p + N;
  *val = x.sws().buf.p + BCG_VECS * N;
}

// the YEqn rows the production path writes straight from the assembly (y_assemble_ell), rebuilt here
// from the LDU matrices by the generic fold (k_ell_build) -- the inspection path the parity tests
// compare the fused kernel against
void bicg_rows_from_ldu_Y(Ctx& x) {
  std::vector<int> map;
  for (int s = 0; s < x.S; ++s) if (s != x.inert) map.push_back(s);
  const int nsys = (int)map.size();
  double *val, *dS, *rhs;
  bicg_layout(x, nsys, &val, &dS, &rhs);
  const long C = x.C, Ce = (long)x.C + x.H;
  x.sws().sysmap.upload(map.data(), nsys, x.stream);
  Matrix& A = x.mY;
  Sys q{A.lower, A.upper, A.diag, A.source, A.ic, A.bc, x.Fs, x.Fs, C, C, x.B, x.f("Y"), C};
  const int nblk = std::min(blocks_for(C, TPB), MAX_BLOCKS);
  hipLaunchKernelGGL(k_ell_build, dim3(nblk, nsys), dim3(TPB), 0, x.stream, x.view(), x.st("Y"), q,
                     (const int*)x.sws().sysmap.p, x.ell.W, x.ell.src.p, Ce, val, dS, rhs, 0,
                     x.ell.eo ? (const int*)x.ell.eo_pos.p : nullptr);
  DFMI_HIP(hipGetLastError());
}

// copy part ("val" [nsys][W][C], "dS" / "rhs" [nsys][C]) of the BiCGStab rows of nsys systems to the host
void bicg_rows_get(Ctx& x, int nsys, const std::string& part, double* host, long count) {
  double *val, *dS, *rhs;
  bicg_layout(x, nsys, &val, &dS, &rhs);
  const long C = x.C, Ce = (long)x.C + x.H;
  const int W = x.ell.W;
  if (part == "val") {
    DFMI_CHECK(count == (long)nsys * W * C, "solver rows: 'val' holds nsys * W * C values");
    DFMI_HIP(hipMemcpyAsync(host, val, count * sizeof(double), hipMemcpyDeviceToHost, x.stream));
  } else {
    DFMI_CHECK(part == "dS" || part == "rhs", "solver rows: part is 'val', 'dS' or 'rhs'");
    DFMI_CHECK(count == (long)nsys * C, "solver rows: 'dS' / 'rhs' hold nsys * C values");
    const double* src = part == "dS" ? dS : rhs;
    for (int s = 0; s < nsys; ++s)
      DFMI_HIP(hipMemcpyAsync(host + (long)s * C, src + s * Ce, C * sizeof(double), hipMemcpyDeviceToHost, x.stream));
  }
  DFMI_HIP(hipStreamSynchronize(x.stream));
  if (x.ell.eo) {   // rows stored colour by colour: back to cell order
    const std::vector<int>& pos = x.ell.h_eo_pos;
    std::vector<double> tmp(C);
    const long nrow = count / C;
    for (long r = 0; r < nrow; ++r) {
      double* h = host + r * C;
      for (int c = 0; c < C; ++c) tmp[c] = h[pos[c]];
      std::copy(tmp.begin(), tmp.end(), h);
    }
  }
}

double solver_work(Ctx& x, const std::string& eqn, bool reset) {
  const int k = work_slot(eqn);
  if (x.work.n == 0) return 0.0;
  double v = 0.0;
  DFMI_HIP(hipMemcpyAsync(&v, x.work.p + k, sizeof(double), hipMemcpyDeviceToHost, x.stream));
  DFMI_HIP(hipStreamSynchronize(x.stream));
  if (reset) {
    DFMI_HIP(hipMemsetAsync(x.work.p + k, 0, sizeof(double), x.stream));
    DFMI_HIP(hipStreamSynchronize(x.stream));
  }
  return v;
}

SolveStats solve_stats(Ctx& x, const std::string& eqn) {
  auto it = x.stat_snap.find(eqn);
  DFMI_CHECK(it != x.stat_snap.end(), "no solve recorded for " + eqn);
  DFMI_HIP(hipStreamSynchronize(x.stream));
  SolveStats st;
  for (int s = 0; s < it->second.nsys; ++s) {   // worst system
    const double* h = it->second.h.p + s * NSCAL;
    st.iters = std::max(st.iters, (int)h[7]);
    st.res0 = std::max(st.res0, h[4]);
    st.res = std::max(st.res, h[4] > 0 ? h[5] / h[4] : 0.0);
  }
  return st;
}

SolveStats solve_bicgstab(Ctx& x, const char* eqn, int nsys, const int* sys_map_host, const double* lower, long lstride,
                          const double* upper, long ustride, const double* diag, long dstride, const double* source,
                          long sstride, const double* ic, const double* bc, long bstride, const char* type_field,
                          double* xsol, long xstride, const SolverCfg& cfg, bool prebuilt) {
  {
    double *v_, *d_, *r_;
    bicg_layout(x, nsys, &v_, &d_, &r_);
  }
  CommTag _ct(x, std::string("bicgstab ") + eqn);
  const long C = x.C, Ce = (long)x.C + x.H;
  const int W = x.ell.W;
  const int nblk = std::min(blocks_for(C, TPB), MAX_BLOCKS);
  auto& WS = x.sws();
  if (WS.scal.n < (size_t)nsys * NSCAL) WS.scal.alloc((size_t)nsys * NSCAL);
  const int* smap = nullptr;
  if (sys_map_host) {
    WS.sysmap.upload(sys_map_host, nsys, x.stream);
    smap = WS.sysmap.p;
  }
  const long N = nsys * Ce;
  double* base = WS.buf.p;
  // U's three components share one operator: built and read once (k_ell_build vshared). Valid because every
  // coupled patch this library accepts is translational (cyclic / processor / processorCyclic: the generic
  // "coupled" code and rotational transforms are rejected at dfmi_set_patch_types), so the coupled-slot
  // coefficients -boundaryCoeffs do not depend on the vector component
  const int vshared = (!prebuilt && nsys > 1 && lstride == 0 && ustride == 0 && std::string(eqn) == "U") ? 1 : 0;
  BV b{base, base + N, base + 2 * N, base + 3 * N, base + 4 * N, base + 5 * N, base + 6 * N, base + 7 * N,
       base + 8 * N, vshared};
  double* val = base + BCG_VECS * N;
  // one partial buffer per reduction site (a converged system's last sums stay intact)
  double* pR = val + (size_t)nsys * W * C;          // (||D r||^2, rho0 | 0): init, xp
  double* pV = pR + (size_t)nsys * nblk * 2;        // r0.v (x 2: the overlapped SpMV's two row sets)
  double* pT = pV + (size_t)nsys * nblk * 2;        // (t.s, t.t, r0.t, r0.s) (x 2 likewise)
  Sys q{lower, upper, diag, source, ic, bc, lstride, ustride, dstride, sstride, bstride, xsol, xstride};
  MeshView m = x.view();
  const int8_t* ty = x.st(type_field);
  dim3 g(nblk, nsys), bl(TPB);
  Launch L{x, nblk, nsys};
  const int* eopos = x.ell.eo ? (const int*)x.ell.eo_pos.p : nullptr;   // rows colour by colour (even-odd)
  if (!prebuilt) {
    KScope _ks(x, "k_ell_build");
    hipLaunchKernelGGL(k_ell_build, g, bl, 0, x.stream, m, ty, q, smap, W, x.ell.src.p, Ce, val, b.dS, b.rhs, vshared,
                       eopos);
  }
  { KScope _ks(x, "k_copy_x"); hipLaunchKernelGGL(k_copy_x, g, bl, 0, x.stream, C, Ce, q, smap, b.xw, eopos); }
  DFMI_HIP(hipGetLastError());
  if (x.ell.eo) {   // the reduced system (build_ell decided; several ranks: split-vector halos, gathered sums)
    const int ne = x.ell.ne, no = (int)C - ne;
    const int hb = std::min(blocks_for(std::max(ne, no), TPB), eo_max_blocks());
    const dim3 gh(hb, nsys);
    const ColView ec = x.ell.eo_cols();
    double* pI = val + (size_t)nsys * W * C;       // (||b - A x0||^2 colour 0)
    double* pR3 = pI + (size_t)nsys * hb;          // (||b - A x0||^2 colour 1, ||D r||^2, r0.r)
    double* pR = pR3 + (size_t)nsys * hb * 3;      // (||D r||^2, 0): the update
    double* pV = pR + (size_t)nsys * hb * 2;       // r0.v
    double* pT = pV + (size_t)nsys * hb;           // (t.s, t.t, r0.t, r0.s)
    // exchange points (several ranks): every kernel that gathers across a processor face reads the other
    // colour's rows of the vector it gathers, exchanged just before it -- only that colour's faces (k: the colour
    // the sending side's cells have, i.e. the colour the half-row pass after it reads)
    auto hx = [&](std::initializer_list<double*> v, int k) { halo_vecs(x, v, nsys, Ce, true, k); };
    hx({b.xw}, -1);   // both halves: init_e reads x's colour 1, init_o its colour 0
    dispatch_W(W, [&](auto wt) {
      constexpr int WT = decltype(wt)::value;
      KScope _ks(x, "k_bcg_init");
      hipLaunchKernelGGL(k_eo_init_e<WT>, gh, bl, 0, x.stream, C, Ce, ne, W, ec, val, b, pI);
    });
    const Red rI = L.after(pI, 1, 1, hb);
    hx({b.p}, 0);
    dispatch_W(W, [&](auto wt) {
      constexpr int WT = decltype(wt)::value;
      KScope _ks(x, "k_bcg_init");
      hipLaunchKernelGGL(k_eo_init_o<WT>, gh, bl, 0, x.stream, C, Ce, ne, no, W, ec, val, b, pR3);
    });
    DFMI_HIP(hipGetLastError());
    Red red = L.after(pR3, 3, 0, hb);
    Poller poll(x, WS.scal.p, nsys, std::string(eqn) + (x.ws_is_y ? "/y" : ""));
    // several ranks: from the second iteration on, ||D r|| of the last update rides the r0.v all-gather and the
    // stop test runs in k_eo_c (two all-gathers per iteration instead of three); the last allowed iteration keeps
    // the test in k_eo_a so the solve ends with its residual recorded
    const bool merged = x.nranks > 1;
    for (int it = 0;; ++it) {
      const bool last = it >= cfg.max_iter;
      const int defer = merged && it > 0 && !last ? 1 : 0;
      if (merged && it > 0 && last) red = L.after(pR, 2, 0, hb);
      hx({b.p}, 1);
      dispatch_W(W, [&](auto wt) {
        constexpr int WT = decltype(wt)::value;
        KScope _ks(x, "k_bcg_eo");
        hipLaunchKernelGGL(k_eo_a<WT>, gh, bl, 0, x.stream, C, Ce, ne, W, ec, val, it, cfg.max_iter, cfg.tol,
                           cfg.abs_tol, rI, red, WS.scal.p, b, defer);
      });
      if (last) break;
      hx({b.p}, 0);   // w in p's colour-0 half
      dispatch_W(W, [&](auto wt) {
        constexpr int WT = decltype(wt)::value;
        KScope _ks(x, "k_bcg_eo");
        hipLaunchKernelGGL(k_eo_b<WT>, gh, bl, 0, x.stream, C, Ce, ne, no, W, ec, val, WS.scal.p, b, pV);
      });
      Red rV;
      if (defer) {   // (r0.v, ||D r||^2) per system in one all-gather
        const size_t per = (size_t)nsys * 4;
        if (WS.red_local.n < 2 * per) WS.red_local.alloc(2 * per);
        if (WS.red_all.n < 2 * per * x.nranks) WS.red_all.alloc(2 * per * x.nranks);
        hipLaunchKernelGGL(k_red_vr, dim3(nsys), dim3(TPB), 0, x.stream, pV, pR, hb, WS.red_local.p);
        DFMI_HIP(hipGetLastError());
        halo_allgather(x, WS.red_local.p, WS.red_all.p, (long)nsys * 2);
        rV = Red{WS.red_all.p, x.nranks, (long)nsys * 2, 2};
      } else {
        rV = L.after(pV, 1, 0, hb);
      }
      hx({b.r, b.v}, 1);
      dispatch_W(W, [&](auto wt) {
        constexpr int WT = decltype(wt)::value;
        KScope _ks(x, "k_bcg_eo");
        hipLaunchKernelGGL(k_eo_c<WT>, gh, bl, 0, x.stream, C, Ce, ne, W, ec, val, rV, WS.scal.p, b, defer, it, cfg.tol,
                           cfg.abs_tol);
      });
      hx({b.t}, 0);   // w2 in t's colour-0 half
      dispatch_W(W, [&](auto wt) {
        constexpr int WT = decltype(wt)::value;
        KScope _ks(x, "k_bcg_eo");
        hipLaunchKernelGGL(k_eo_d<WT>, gh, bl, 0, x.stream, C, Ce, ne, no, W, ec, val, WS.scal.p, b, pT);
      });
      const Red rT = L.after(pT, 4, 0, hb);
      const long long pseq = poll.plan(it);   // the update kernel posts this iteration's record (no extra launch)
      { KScope _ks(x, "k_bcg_xp"); hipLaunchKernelGGL(k_eo_xp, gh, bl, 0, x.stream, Ce, ne, no, rT, WS.scal.p, b, pR,
                                                      pseq ? WS.poll.d : (PollRec*)nullptr, pseq); }
      DFMI_HIP(hipGetLastError());
      if (!merged) red = L.after(pR, 2, 0, hb);
      if (poll.check()) break;
    }
    hx({b.xw}, 1);
    dispatch_W(W, [&](auto wt) {
      constexpr int WT = decltype(wt)::value;
      KScope _ks(x, "k_eo_final");
      hipLaunchKernelGGL(k_eo_final<WT>, gh, bl, 0, x.stream, C, Ce, ne, no, W, ec, val, WS.scal.p, b, q, smap,
                         (const int*)x.ell.eo_cell.p);
    });
    DFMI_HIP(hipGetLastError());
    record_stats(x, eqn, WS.scal.p, nsys);
    return SolveStats{};
  }
  halo_vecs(x, {b.xw}, nsys, Ce);
  if (small_solve(x)) {
    dispatch_W(W, [&](auto wt) {
      constexpr int WT = decltype(wt)::value;
      KScope _ks(x, "k_bcg_small");
      hipLaunchKernelGGL(k_bcg_small<WT>, dim3(nsys), dim3(STPB), 0, x.stream, C, Ce, W, x.ell.col.p, val, cfg.max_iter,
                         cfg.tol, cfg.abs_tol, WS.scal.p, b, q, smap);
    });
    DFMI_HIP(hipGetLastError());
    record_stats(x, eqn, WS.scal.p, nsys);
    return SolveStats{};
  }
  dispatch_W(W, [&](auto wt) {
    constexpr int WT = decltype(wt)::value;
    { KScope _ks(x, "k_bcg_init"); hipLaunchKernelGGL(k_bcg_init<WT>, g, bl, 0, x.stream, C, Ce, W, x.ell.cols(), val, b, pR); }
  });
  DFMI_HIP(hipGetLastError());
  Red red = L.after(pR, 2);
  Poller poll(x, WS.scal.p, nsys, std::string(eqn) + (x.ws_is_y ? "/y" : ""));
  for (int it = 0;; ++it) {
    const int np1 = spmv_with_halo(x, {b.p}, nsys, Ce, nblk, [&](RowSet rs) {
      dispatch_W(W, [&](auto wt) {
        constexpr int WT = decltype(wt)::value;
        KScope _ks(x, "k_bcg_spmv");
        hipLaunchKernelGGL((k_bcg_spmv1<WT>), g, bl, 0, x.stream, C, Ce, W, x.ell.cols(), val, it, cfg.max_iter,
                           cfg.tol, cfg.abs_tol, red, WS.scal.p, b, pV, rs);
      });
    });
    if (it >= cfg.max_iter) break;
    red = L.after(pV, 1, 0, np1);
    // processor neighbours read s from the exchanged sv
    if (halo_active(x)) { KScope _ks(x, "k_bcg_s"); hipLaunchKernelGGL(k_bcg_s, g, bl, 0, x.stream, C, Ce, red, WS.scal.p, b); }
    const int np2 = spmv_with_halo(x, {b.sv}, nsys, Ce, nblk, [&](RowSet rs) {
      dispatch_W(W, [&](auto wt) {
        constexpr int WT = decltype(wt)::value;
        KScope _ks(x, "k_bcg_spmv");
        hipLaunchKernelGGL((k_bcg_spmv2<WT>), g, bl, 0, x.stream, C, Ce, W, x.ell.cols(), val, red, WS.scal.p, b, pT, rs);
      });
    });
    const Red red_t = L.after(pT, 4, 0, np2);
    { KScope _ks(x, "k_bcg_xp"); hipLaunchKernelGGL(k_bcg_xp, g, bl, 0, x.stream, C, Ce, red_t, q, smap, WS.scal.p, b, pR); }
    DFMI_HIP(hipGetLastError());
    red = L.after(pR, 2, 0);
    if (poll.after(it)) break;
  }
  DFMI_HIP(hipGetLastError());
  record_stats(x, eqn, WS.scal.p, nsys);
  return SolveStats{};
}

SolveStats solve_pcg(Ctx& x, const char* eqn, const double* lower, const double* upper, const double* diag,
                     const double* source, const double* ic, const double* bc, const char* type_field, double* xsol,
                     double* bxsol, const SolverCfg& cfg) {
  (void)bxsol;
  if (!x.ell.ready) build_ell(x);
  CommTag _ct(x, std::string("pcg ") + eqn);
  const long C = x.C, Ce = (long)x.C + x.H;
  const int W = x.ell.W;
  const int nblk = std::min(blocks_for(C, TPB), cg_max_blocks());
  auto& WS = x.sws();
  const size_t need = 8 * Ce + (size_t)W * C + (size_t)nblk * 6 + 64;
  if (WS.buf.n < need) WS.buf.alloc(need);
  if (WS.scal.n < NSCAL) WS.scal.alloc(NSCAL);
  double* base = WS.buf.p;
  CV v{base, base + Ce, base + 2 * Ce, base + 3 * Ce, base + 4 * Ce, base + 5 * Ce, base + 6 * Ce, base + 7 * Ce};
  double* val = base + 8 * Ce;
  double* q1 = val + (size_t)W * C;    // p.q
  double* q2 = q1 + (size_t)nblk * 2;  // (r.z [Jacobi], r.r); q1 holds 2 nblk for the overlapped SpMV
  double* q3 = q2 + (size_t)nblk * 2;  // r.z (AMG)
  Sys q{lower, upper, diag, source, ic, bc, 0, 0, 0, 0, 0, xsol, 0};
  MeshView m = x.view();
  const int8_t* ty = x.st(type_field);
  dim3 g(nblk), bl(TPB);
  Launch L{x, nblk, 1};
  const bool amg = cfg.precond == 1;
  // the symmetric p operator read face-wise on a hex box (FaceOp, one rank; pcg.face_form = 0: the ELL values)
  const bool face = x.hex[0] > 0 && x.fslot && x.nranks == 1 && !halo_active(x) && !small_solve(x) && x.on("pcg.face_form");
  // a later corrector of the same step (amg.reuse): the V-cycle keeps the operators the first corrector built --
  // a fixed SPD preconditioner of a matrix that changed by the density update only, so PCG still converges to
  // this system's own tolerance; the fp32 rounding and Galerkin sums of one solve are saved
  const bool reuse = amg && x.amg.ready && x.amg.reuse_ok && x.on("amg.reuse") && x.nranks == 1;
  // face-wise PCG with the reused V-cycle: nothing reads the ELL values, so they are not written -- only when
  // the V-cycle's level 0 is the face-wise fp32 copy too (the fp64 V-cycle's level 0 reads the ELL values of
  // THIS solve beside its diagonal, so they must be current)
  const int novals = face && reuse && amg_l0_fusable(x) ? 2 : 0;
  { KScope _ks(x, "k_ell_build"); hipLaunchKernelGGL(k_ell_build, g, bl, 0, x.stream, m, ty, q, (const int*)nullptr, W, x.ell.src.p, Ce, val, v.dS, v.rhs, novals); }
  { KScope _ks(x, "k_copy_x"); hipLaunchKernelGGL(k_copy_x, g, bl, 0, x.stream, C, Ce, q, (const int*)nullptr, v.xw); }
  DFMI_HIP(hipGetLastError());
  FaceOp<double> fo{};
  if (face) fo = FaceOp<double>{1, x.hex[0], x.hex[1], x.hex[2], C, upper, bc, x.ell.csStart.p, x.ell.csSlot.p,
                                x.ell.scol.p};
  if (amg) {
    if (!x.amg.ready) amg_setup(x);
    x.amg.face = face && amg_l0_fusable(x) && x.amg.l0_sweeps == 1;
    x.amg.dfo = fo;
    if (!reuse) amg_galerkin(x, val, v.dS);
    if (x.amg.halo_l0) {   // the level-0 diagonal across processor faces, once per solve
      halo_vecs(x, {v.dS}, 1, Ce);
      x.amg.dS_full = v.dS;
    }
  }
  halo_vecs(x, {v.xw}, 1, Ce);
  if (small_solve(x)) {
    dispatch_W(W, [&](auto wt) {
      constexpr int WT = decltype(wt)::value;
      KScope _ks(x, "k_pcg_small");
      if (!amg) {
        AmgView<double> none{};
        hipLaunchKernelGGL((k_pcg_small<WT, double, false>), dim3(1), dim3(STPB), 0, x.stream, C, W, x.ell.col.p, val,
                           cfg.max_iter, cfg.tol, cfg.abs_tol, WS.scal.p, v, xsol, none);
      } else if (x.amg.fp32) {
        hipLaunchKernelGGL((k_pcg_small<WT, float, true>), dim3(1), dim3(STPB), 0, x.stream, C, W, x.ell.col.p, val,
                           cfg.max_iter, cfg.tol, cfg.abs_tol, WS.scal.p, v, xsol, amg_view_f32(x, x.ell.col.p));
      } else {
        hipLaunchKernelGGL((k_pcg_small<WT, double, true>), dim3(1), dim3(STPB), 0, x.stream, C, W, x.ell.col.p, val,
                           cfg.max_iter, cfg.tol, cfg.abs_tol, WS.scal.p, v, xsol, amg_view_f64(x, val, v.dS, x.ell.col.p));
      }
    });
    DFMI_HIP(hipGetLastError());
    record_stats(x, eqn, WS.scal.p, 1);
    return SolveStats{};
  }
  dispatch_W(W, [&](auto wt) {
    constexpr int WT = decltype(wt)::value;
    KScope _ks(x, "k_cg_init");
    if (face) hipLaunchKernelGGL((k_cg_init<0, true>), g, bl, 0, x.stream, C, W, x.ell.cols(), val, v, q2, fo);
    else hipLaunchKernelGGL(k_cg_init<WT>, g, bl, 0, x.stream, C, W, x.ell.cols(), val, v, q2, fo);
  });
  DFMI_HIP(hipGetLastError());
  if (x.nranks > 1) {
    // several ranks: the single-reduction form -- per iteration the preconditioner, w = A z with z's halo, and ONE
    // all-gather of (||r||^2, r.z, z.w), then the update (two all-gathers and the p_old halo in the standard form)
    if (x.sws().red_local.n < 8) x.sws().red_local.alloc(8);
    if (x.sws().red_all.n < (size_t)8 * x.nranks) x.sws().red_all.alloc((size_t)8 * x.nranks);
    double* loc = x.sws().red_local.p;
    double* all = x.sws().red_all.p;
    const Red red_g{all, x.nranks, 3, 0};
    Poller poll(x, WS.scal.p, 1, std::string(eqn) + (amg ? "/amg" : "/jacobi") + "/cg1");
    for (int it = 0;; ++it) {
      if (amg) {
        if (x.amg.halo_l0) halo_vecs(x, {v.r}, 1, Ce);   // the V-cycle's level 0 reads the residual across ranks
        amg_apply(x, val, v.dS, x.ell.cols(), v.r, v.z, q3, nblk, it == 0 ? nullptr : WS.scal.p + 6);
      }
      const int np = spmv_with_halo(x, {v.z}, 1, Ce, nblk, [&](RowSet rs) {
        dispatch_W(W, [&](auto wt) {
          constexpr int WT = decltype(wt)::value;
          KScope _ks(x, "k_cg_spmv");
          hipLaunchKernelGGL(k_cgcg_w<WT>, g, bl, 0, x.stream, C, W, x.ell.cols(), val, WS.scal.p, it, v, q1, rs);
        });
      });
      hipLaunchKernelGGL(k_cgcg_local, dim3(1), dim3(TPB), 0, x.stream, Red{q2 + 1, nblk, 2, 0},
                         amg ? Red{q3, nblk, 1, 0} : Red{q2, nblk, 2, 0}, Red{q1, np, 1, 0}, WS.scal.p, it, loc);
      DFMI_HIP(hipGetLastError());
      halo_allgather(x, loc, all, 3);
      {
        KScope _ks(x, "k_cg_x");
        if (amg)
          hipLaunchKernelGGL(k_cgcg_update<false>, g, bl, 0, x.stream, C, it, cfg.max_iter, cfg.tol, cfg.abs_tol, red_g,
                             WS.scal.p, xsol, v, q2);
        else
          hipLaunchKernelGGL(k_cgcg_update<true>, g, bl, 0, x.stream, C, it, cfg.max_iter, cfg.tol, cfg.abs_tol, red_g,
                             WS.scal.p, xsol, v, q2);
      }
      DFMI_HIP(hipGetLastError());
      if (it >= cfg.max_iter) break;
      if (poll.after(it)) break;
    }
    record_stats(x, eqn, WS.scal.p, 1);
    return SolveStats{};
  }
  // (r.z, r.r) readers: Jacobi -> both from q2; AMG -> r.z from the V-cycle's partials in q3
  // act: the solve's active flag (after the first iteration the V-cycle of a stopped solve is skipped)
  auto reds = [&](Red& rz, Red& rr, const double* act) {   // one rank (several ranks: the form above)
    Red r2 = L.after(q2, 2, 0);
    rr = r2; rr.p += 1;
    if (amg) {
      amg_apply(x, val, v.dS, x.ell.cols(), v.r, v.z, q3, nblk, act);
      rz = L.after(q3, 1, 1);
    } else rz = r2;
  };
  Red red_rz, red_rr;
  reds(red_rz, red_rr, nullptr);
  Poller poll(x, WS.scal.p, 1, std::string(eqn) + (amg ? "/amg" : "/jacobi"));
  double* pold = v.pa;
  double* pnew = v.pb;
  // one rank: the update kernel also does the V-cycle's level-0 first sweep (pcg.fuse_l0 = 0: separate)
  const bool fuse_l0 = amg && x.nranks == 1 && !halo_active(x) && amg_l0_fusable(x) && x.on("pcg.fuse_l0");
  for (int it = 0;; ++it) {
    const int np = spmv_with_halo(x, {v.z, pold}, 1, Ce, nblk, [&](RowSet rs) {
      dispatch_W(W, [&](auto wt) {
        constexpr int WT = decltype(wt)::value;
        KScope _ks(x, "k_cg_spmv");
        if (face)
          hipLaunchKernelGGL((k_cg_spmv<0, true>), g, bl, 0, x.stream, C, W, x.ell.cols(), val, it, cfg.max_iter,
                             cfg.tol, cfg.abs_tol, red_rz, red_rr, WS.scal.p, v, pold, pnew, q1, rs, fo);
        else
          hipLaunchKernelGGL(k_cg_spmv<WT>, g, bl, 0, x.stream, C, W, x.ell.cols(), val, it, cfg.max_iter, cfg.tol,
                             cfg.abs_tol, red_rz, red_rr, WS.scal.p, v, pold, pnew, q1, rs, fo);
      });
    });
    if (it >= cfg.max_iter) break;
    Red red = L.after(q1, 1, 0, np);
    if (fuse_l0) {
      AmgLevel& l0 = x.amg.lv[0];
      dispatch_W(W, [&](auto wt) {
        constexpr int WT = decltype(wt)::value;
        KScope _ks(x, "k_cg_x_smooth");   // its own timer name: tests assert the fused path ran
        if (x.amg.face)
          hipLaunchKernelGGL((k_cg_x_smooth<0, float, true>), g, bl, 0, x.stream, C, W, x.ell.cols(), red, WS.scal.p,
                             xsol, v, pnew, v.z, q2, (const float*)l0.fval.p, (const float*)l0.fD.p, (float)x.amg.omega,
                             l0.fx.p, l0.fr.p, x.amg.ffo);
        else
          hipLaunchKernelGGL((k_cg_x_smooth<WT, float>), g, bl, 0, x.stream, C, W, x.ell.cols(), red, WS.scal.p, xsol,
                             v, pnew, v.z, q2, (const float*)l0.fval.p, (const float*)l0.fD.p, (float)x.amg.omega,
                             l0.fx.p, l0.fr.p, x.amg.ffo);
      });
      DFMI_HIP(hipGetLastError());
      std::swap(v.r, v.z);   // z was dead (k_cg_spmv has read it); the V-cycle writes the new z over the old r
      Red r2 = L.after(q2, 2, 0);
      red_rr = r2; red_rr.p += 1;
      // the next iteration's stop test runs in the V-cycle's first launch (CgStop): no V-cycle after convergence
      amg_apply(x, val, v.dS, x.ell.cols(), v.r, v.z, q3, nblk, WS.scal.p + 6, true,
                CgStop{red_rr, WS.scal.p, it + 1, cfg.tol, cfg.abs_tol});
      red_rz = L.after(q3, 1, 1);
      std::swap(pold, pnew);
      if (poll.after(it)) break;
      continue;
    }
    {
      KScope _ks(x, "k_cg_x");
      if (amg) hipLaunchKernelGGL(k_cg_x<false>, g, bl, 0, x.stream, C, red, WS.scal.p, xsol, v, pnew, q2);
      else hipLaunchKernelGGL(k_cg_x<true>, g, bl, 0, x.stream, C, red, WS.scal.p, xsol, v, pnew, q2);
    }
    DFMI_HIP(hipGetLastError());
    reds(red_rz, red_rr, WS.scal.p + 6);
    std::swap(pold, pnew);
    if (poll.after(it)) break;
  }
  DFMI_HIP(hipGetLastError());
  record_stats(x, eqn, WS.scal.p, 1);
  return SolveStats{};
}

}  // namespace dfmi
