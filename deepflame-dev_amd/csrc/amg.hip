// amg.hip -- aggregation-AMG V-cycle preconditioner for the pressure PCG (replaces AmgX's
// AGGREGATION / V-cycle p solver, reference examples/.../system/amgxpOptions:1-18,
// src_gpu/AmgXSolver.cu:184-340).
//
// Hierarchy (built once per mesh on the host, since it depends only on geometry): three greedy
// pairwise-matching passes per level on the strength graph |Sf| * deltaCoeffs (the geometric part
// of the laplacian coefficients), so a uniform hex mesh coarsens 2x2x2 per level (AmgX SIZE_2
// selector, applied three times). Aggregates never cross ranks: the preconditioner is rank-local
// (block-Jacobi across processor faces); the outer PCG SpMV carries the halo.
// Per solve: Galerkin coarse operators P^T A P (piecewise-constant P) are summed on the device from
// precomputed contribution lists in a fixed order -- deterministic, no atomics.
// V-cycle: one weighted-Jacobi pre-sweep from zero (fused into the residual pass), restriction,
// coarse correction scaled by an over-correction factor (1.35: piecewise-constant interpolation
// under-corrects smooth errors; 28 instead of 32 PCG iterations per 2M-cell step), prolongation fused
// with one post-sweep; the coarsest level (<= 4096 cells) is
// smoothed by a fixed number of Jacobi sweeps inside one workgroup (LDS-resident vectors). All pieces
// are linear and the pre/post sweeps are adjoint, so the preconditioner is symmetric (valid for CG).
// Precision: by default the whole V-cycle runs in fp32 (operators rounded once per solve, work
// vectors in float; AmgX's mixed-precision mode) -- it only preconditions, the PCG residuals, dot
// products and solution stay fp64 -- which halves the preconditioner's bytes per iteration.
#include "dfmi_ctx.h"
#include "amg.h"
#include "amg_graph.h"
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <numeric>
#include <string>
#include <type_traits>

namespace dfmi {
namespace {

constexpr int TPB = 256;
constexpr int COARSEST = 1024;   // k_coarsest capacity (cells); also n * W <= LDS_ENT
constexpr int CTPB = 1024;

// ---------------------------------------------------------------- kernels
// Value type T is the V-cycle precision (double, or float in the default mixed mode); TB the type
// of a level's right-hand side (level 0: the PCG residual, always double); TO the type written out.

// coarse values: out[s * nc + I] = sum (in double) of the fine sources listed for (slot s, cell I); one
// thread per (slot, cell) entry, so a cell's lists are walked in parallel rather than one after another
template <class TF, class TC>
__global__ void k_galerkin(int nc, int slots, const int* __restrict__ gstart, const int* __restrict__ gsrc,
                           const TF* __restrict__ fval, const TF* __restrict__ fD, TC* __restrict__ cval,
                           TC* __restrict__ cD) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)nc * slots) return;
  const int s = (int)(t / nc), I = (int)(t % nc);
  const long e0 = gstart[t], e1 = gstart[t + 1];
  double a = 0.0;
  for (long e = e0; e < e1; ++e) {
    const int src = gsrc[e];
    a += src >= 0 ? (double)fval[src] : (double)fD[-src - 1];
  }
  if (s < slots - 1) cval[t] = (TC)a;
  else cD[I] = e0 == e1 ? (TC)1 : (TC)a;   // an empty (padding) cell of a padded level: unit diagonal
}

// level-0 operator rounded to the V-cycle precision (once per solve)
__global__ void k_round_f32(long n, const double* __restrict__ a, float* __restrict__ b) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) b[i] = (float)a[i];
}

// x = omega b / D (first sweep from zero); r = b - A x   (columns >= n: other ranks, dropped)
template <int WT, class T, class TB, bool FF = false>
__global__ void __launch_bounds__(TPB) k_smooth_res(int n, int W_, ColView col,
                                                    const T* __restrict__ val, const T* __restrict__ D,
                                                    const TB* __restrict__ b, T omega,
                                                    T* __restrict__ x, T* __restrict__ r, const double* act,
                                                    FaceOp<T> fo = {}) {
  __shared__ int s_ct[CT_MAX];
  if (!FF) col.stage(s_ct);
  const int W = WT > 0 ? WT : W_;
  const int c = xcd_block() * blockDim.x + threadIdx.x;
  if (c >= n || (act && *act == 0.0)) return;
  const T bc = (T)b[c];
  const T xc = omega * bc / D[c];
  T y = D[c] * xc;
  if constexpr (FF) {
    face_row(fo, c, [&](int j, T a) { if (j < n) y += a * (omega * (T)b[j] / D[j]); });
  } else {
    const int rb = col.row(c);
#pragma unroll
    for (int k = 0; k < W; ++k) {
      const int j = col.get(s_ct, rb, n, k, c);
      if (j < n) y += val[(long)k * n + c] * (omega * (T)b[j] / D[j]);
    }
  }
  x[c] = xc;
  r[c] = bc - y;
}

// a further level-0 pre-sweep (amg.presweeps > 1): x += omega r / D, r_new = r - A (omega r / D)
template <int WT, class T>
__global__ void __launch_bounds__(TPB) k_smooth_step(int n, int W_, ColView col,
                                                     const T* __restrict__ val, const T* __restrict__ D,
                                                     const T* __restrict__ r, T omega, T* __restrict__ x,
                                                     T* __restrict__ rn, const double* act) {
  __shared__ int s_ct[CT_MAX];
  col.stage(s_ct);
  const int W = WT > 0 ? WT : W_;
  const int c = xcd_block() * blockDim.x + threadIdx.x;
  if (c >= n || (act && *act == 0.0)) return;
  const T rc = r[c];
  const T dc = omega * rc / D[c];
  T y = D[c] * dc;
  const int rb = col.row(c);
#pragma unroll
  for (int k = 0; k < W; ++k) {
    const int j = col.get(s_ct, rb, n, k, c);
    if (j < n) y += val[(long)k * n + c] * (omega * r[j] / D[j]);
  }
  x[c] += dc;
  rn[c] = rc - y;
}

// a further level-0 post-sweep: out = in + omega (b - A in) / D; optional block partials of b.out
template <int WT, class T, class TB, class TO>
__global__ void __launch_bounds__(TPB) k_jacobi_sweep(int n, int W_, ColView col,
                                                      const T* __restrict__ val, const T* __restrict__ D,
                                                      const TB* __restrict__ b, const TO* __restrict__ in, T omega,
                                                      TO* __restrict__ out, double* partial, const double* act) {
  __shared__ int s_ct[CT_MAX];
  col.stage(s_ct);
  const int W = WT > 0 ? WT : W_;
  if (act && *act == 0.0) return;
  __shared__ double sh[TPB / 64];
  double acc = 0.0;
  for (int c = xcd_block() * blockDim.x + threadIdx.x; c < n; c += gridDim.x * blockDim.x) {
    const T yc = (T)in[c];
    T ay = D[c] * yc;
  const int rb = col.row(c);
#pragma unroll
    for (int k = 0; k < W; ++k) {
      const int j = col.get(s_ct, rb, n, k, c);
      if (j < n) ay += val[(long)k * n + c] * (T)in[j];
    }
    const TB bc = b[c];
    const TO o = (TO)(yc + omega * ((T)bc - ay) / D[c]);
    out[c] = o;
    acc += (double)bc * (double)o;
  }
  if (!partial) return;
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0;
    for (int w = 0; w < TPB / 64; ++w) a += sh[w];
    partial[blockIdx.x] = a;
  }
}

// padded coarse levels (pad_levels): first sweep from zero + residual as k_smooth_res, and the restriction
// to the next level summed over the 8 lanes of the aggregate (in member order, as k_restrict) -- n is a
// multiple of 8 and every aligned group of 8 threads is one aggregate, so a group exits or runs together
template <int WT, class T>
__global__ void __launch_bounds__(TPB) k_smooth_res_r8(int n, int W_, const int* __restrict__ col,
                                                       const T* __restrict__ val, const T* __restrict__ D,
                                                       const T* __restrict__ b, T omega, T* __restrict__ x,
                                                       T* __restrict__ bnext, const double* act) {
  const int W = WT > 0 ? WT : W_;
  const int c = xcd_block() * blockDim.x + threadIdx.x;
  if (c >= n || (act && *act == 0.0)) return;
  const T bc = b[c];
  const T xc = omega * bc / D[c];
  T y = D[c] * xc;
#pragma unroll
  for (int k = 0; k < W; ++k) {
    const int j = col[(long)k * n + c];
    if (j < n) y += val[(long)k * n + c] * (omega * b[j] / D[j]);
  }
  x[c] = xc;
  const T r = bc - y;
  T s = 0;
#pragma unroll
  for (int m = 0; m < 8; ++m) s += __shfl(r, m, 8);
  if ((threadIdx.x & 7) == 0) bnext[c >> 3] = s;
}

// level 0 with its processor couplings (Amg::halo_l0): the first sweep from zero + residual as k_smooth_res,
// the halo columns included -- x0 at a halo cell is omega r_j / D_j from the exchanged residual and diagonal
// (the peer's own x0_j: D_j rounded to T as its level-0 copy is)
template <int WT, class T>
__global__ void __launch_bounds__(TPB) k_smooth_res_h(int n, int W_, ColView col, const T* __restrict__ val,
                                                      const T* __restrict__ D, const double* __restrict__ b,
                                                      const double* __restrict__ dh, T omega, T* __restrict__ x,
                                                      T* __restrict__ r, const double* act) {
  __shared__ int s_ct[CT_MAX];
  col.stage(s_ct);
  const int W = WT > 0 ? WT : W_;
  const int c = xcd_block() * blockDim.x + threadIdx.x;
  if (c >= n || (act && *act == 0.0)) return;
  const T bc = (T)b[c];
  const T xc = omega * bc / D[c];
  T y = D[c] * xc;
  const int rb = col.row(c);
#pragma unroll
  for (int k = 0; k < W; ++k) {
    const int j = col.get(s_ct, rb, n, k, c);
    const T dj = j < n ? D[j] : (T)dh[j];
    y += val[(long)k * n + c] * (omega * (T)b[j] / dj);
  }
  x[c] = xc;
  r[c] = bc - y;
}
// y = x0 + sc P xc on level 0 (the iterate the post-sweep smooths), in double for the halo exchange
template <class T>
__global__ void k_prolong_y(int n, const T* __restrict__ x, const int* __restrict__ agg, const T* __restrict__ xc, T sc,
                            double* __restrict__ y, const double* act) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n || (act && *act == 0.0)) return;
  y[c] = (double)(x[c] + sc * xc[agg[c]]);
}
// the post-sweep with the processor columns: out = y + omega (b - A y) / D, y incl. the exchanged halo;
// block partials of b.out
template <int WT, class T>
__global__ void __launch_bounds__(TPB) k_post_smooth_h(int n, int W_, ColView col, const T* __restrict__ val,
                                                       const T* __restrict__ D, const double* __restrict__ b,
                                                       const double* __restrict__ y, T omega, double* __restrict__ out,
                                                       double* partial, const double* act) {
  __shared__ int s_ct[CT_MAX];
  col.stage(s_ct);
  const int W = WT > 0 ? WT : W_;
  if (act && *act == 0.0) return;
  __shared__ double sh[TPB / 64];
  double acc = 0.0;
  for (int c = xcd_block() * blockDim.x + threadIdx.x; c < n; c += gridDim.x * blockDim.x) {
    const T yc = (T)y[c];
    T ay = D[c] * yc;
    const int rb = col.row(c);
#pragma unroll
    for (int k = 0; k < W; ++k) {
      const int j = col.get(s_ct, rb, n, k, c);
      ay += val[(long)k * n + c] * (T)y[j];
    }
    const double bc = b[c];
    const double o = (double)(yc + omega * ((T)bc - ay) / D[c]);
    out[c] = o;
    acc += bc * o;
  }
  if (!partial) return;
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0;
    for (int w = 0; w < TPB / 64; ++w) a += sh[w];
    partial[blockIdx.x] = a;
  }
}

template <class T>
__global__ void __launch_bounds__(TPB) k_restrict(int nc, const int* __restrict__ mstart, const int* __restrict__ members,
                                                  const T* __restrict__ r, T* __restrict__ bc, const double* act,
                                                  CgStop st = CgStop{}) {
  if (st.scal) {   // every block repeats the PCG stop test (CgStop); block 0 records it
    __shared__ double sa;
    if (threadIdx.x == 0) sa = *act;   // one read per block: block 0 may set the flag meanwhile
    __syncthreads();
    if (sa == 0.0) return;
    double b[1];
    red_sum<1>(st.rr, 0, b);
    const double res = sqrt(b[0]);
    if (res <= st.tol * st.scal[4] || res <= st.abs_tol) {
      if (blockIdx.x == 0 && threadIdx.x == 0) { st.scal[5] = res; st.scal[7] = st.it; st.scal[6] = 0.0; }
      return;
    }
  } else if (act && *act == 0.0) {
    return;
  }
  const int I = blockIdx.x * blockDim.x + threadIdx.x;
  if (I >= nc) return;
  T a = 0;
  for (int e = mstart[I]; e < mstart[I + 1]; ++e) a += r[members[e]];
  bc[I] = a;
}

// y = x + s P xc; out = y + omega (b - A y) / D; optional block partials of b.out (level 0: r.z,
// formed in double from the values actually stored)
template <int WT, class T, class TB, class TO, bool FF = false>
__global__ void __launch_bounds__(TPB) k_prolong_smooth(int n, int W_, ColView col,
                                                        const T* __restrict__ val, const T* __restrict__ D,
                                                        const TB* __restrict__ b, const T* __restrict__ x,
                                                        const int* __restrict__ agg, const T* __restrict__ xc,
                                                        T omega, T sc, TO* __restrict__ out, double* partial,
                                                        const double* act, FaceOp<T> fo = {}) {
  __shared__ int s_ct[CT_MAX];
  if (!FF) col.stage(s_ct);
  const int W = WT > 0 ? WT : W_;
  if (act && *act == 0.0) return;   // uniform: no barrier below is reached by part of the block
  __shared__ double sh[TPB / 64];
  double acc = 0.0;
  for (int c = xcd_block() * blockDim.x + threadIdx.x; c < n; c += gridDim.x * blockDim.x) {
    const T yc = x[c] + sc * xc[agg[c]];
    T ay = D[c] * yc;
    if constexpr (FF) {
      face_row(fo, c, [&](int j, T a) { if (j < n) ay += a * (x[j] + sc * xc[agg[j]]); });
    } else {
      const int rb = col.row(c);
#pragma unroll
      for (int k = 0; k < W; ++k) {
        const int j = col.get(s_ct, rb, n, k, c);
        if (j < n) ay += val[(long)k * n + c] * (x[j] + sc * xc[agg[j]]);
      }
    }
    const TB bc = b[c];
    const TO o = (TO)(yc + omega * ((T)bc - ay) / D[c]);
    out[c] = o;
    acc += (double)bc * (double)o;
  }
  if (!partial) return;
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0;
    for (int w = 0; w < TPB / 64; ++w) a += sh[w];
    partial[blockIdx.x] = a;
  }
}

__global__ void k_dot_partial(int n, const double* __restrict__ a, const double* __restrict__ b, double* partial) {
  __shared__ double sh[TPB / 64];
  double acc = 0.0;
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < n; c += gridDim.x * blockDim.x) acc += a[c] * b[c];
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int w = 0; w < TPB / 64; ++w) s += sh[w];
    partial[blockIdx.x] = s;
  }
}

// coarsest level: `sweeps` weighted-Jacobi sweeps from zero in one workgroup; operator and vectors
// staged in LDS (n * W <= LDS_ENT), so the sweeps run at LDS latency
constexpr int LDS_ENT = 6144;
template <class T, class TB, class TO>
__global__ void __launch_bounds__(CTPB) k_coarsest(int n, int W, const int* __restrict__ col,
                                                   const T* __restrict__ val, const T* __restrict__ D,
                                                   const TB* __restrict__ b, T omega, int sweeps,
                                                   TO* __restrict__ x, const double* act) {
  if (act && *act == 0.0) return;
  __shared__ T xa[COARSEST], xb[COARSEST];
  __shared__ T sv[LDS_ENT];
  __shared__ int sc[LDS_ENT];
  __shared__ T sd[COARSEST], sb[COARSEST];
  for (int e = threadIdx.x; e < n * W; e += CTPB) { sv[e] = val[e]; sc[e] = col[e]; }
  for (int c = threadIdx.x; c < n; c += CTPB) { sd[c] = D[c]; sb[c] = (T)b[c]; xa[c] = omega * (T)b[c] / D[c]; }
  __syncthreads();
  T* cur = xa;
  T* nxt = xb;
  for (int s = 1; s < sweeps; ++s) {
    for (int c = threadIdx.x; c < n; c += CTPB) {
      T y = sd[c] * cur[c];
      for (int k = 0; k < W; ++k) {
        const int j = sc[k * n + c];
        if (j < n) y += sv[k * n + c] * cur[j];
      }
      nxt[c] = cur[c] + omega * (sb[c] - y) / sd[c];
    }
    __syncthreads();
    T* t = cur; cur = nxt; nxt = t;
  }
  for (int c = threadIdx.x; c < n; c += CTPB) x[c] = (TO)cur[c];
}

// The V-cycle's tail in ONE workgroup (Amg::tail): the padded level t = L - 2 (n <= TAIL_N cells, its rows
// held in registers, four cells per thread, its vectors in LDS), its restriction, the coarsest level's sweeps
// (LDS-resident as k_coarsest) and level t's prolongation + post-sweep -- the work of k_smooth_res_r8 +
// k_coarsest + k_prolong_smooth on those levels, with their expressions in their order, so the corrected
// level-t iterate written to xo is bitwise theirs. Three launches of ~6-8 us (latency: a few dependent
// loads each, no bandwidth to speak of on <= 4096 cells) become one.
constexpr int TAIL_N = 4096, TAIL_W = 8;
template <int WT, class T>
__global__ void __launch_bounds__(CTPB) k_vtail(int n, int W_, const int* __restrict__ col, const T* __restrict__ val,
                                                const T* __restrict__ D, const T* __restrict__ b, int nc, int Wc,
                                                const int* __restrict__ colc, const T* __restrict__ valc,
                                                const T* __restrict__ Dc, T omega, T sc, int sweeps,
                                                T* __restrict__ xo, const double* act) {
  if (act && *act == 0.0) return;   // uniform
  const int W = WT > 0 ? WT : W_;
  constexpr int Q = TAIL_N / CTPB;
  __shared__ T sb[TAIL_N], sD[TAIL_N], sx[TAIL_N];
  __shared__ T xa[COARSEST], xb[COARSEST], sdc[COARSEST], sbc[COARSEST];
  __shared__ T sv[LDS_ENT];
  __shared__ int scl[LDS_ENT];
  const int tid = threadIdx.x;
  int cj[Q][TAIL_W];
  T cv[Q][TAIL_W];
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int c = q * CTPB + tid;
    if (c >= n) continue;
    sb[c] = b[c];
    sD[c] = D[c];
#pragma unroll
    for (int k = 0; k < TAIL_W; ++k)
      if (k < W) { cj[q][k] = col[(long)k * n + c]; cv[q][k] = val[(long)k * n + c]; }
  }
  for (int e = tid; e < nc * Wc; e += CTPB) { sv[e] = valc[e]; scl[e] = colc[e]; }
  for (int c = tid; c < nc; c += CTPB) sdc[c] = Dc[c];
  __syncthreads();
  // down: one sweep from zero + residual, summed over each aligned group of 8 (k_smooth_res_r8)
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int c = q * CTPB + tid;
    if (c >= n) continue;   // n % 8 == 0: a group of 8 lanes runs or skips together
    const T bc = sb[c];
    const T xc = omega * bc / sD[c];
    T y = sD[c] * xc;
#pragma unroll
    for (int k = 0; k < TAIL_W; ++k) {
      if (k >= W) break;
      const int j = cj[q][k];
      if (j < n) y += cv[q][k] * (omega * sb[j] / sD[j]);
    }
    sx[c] = xc;
    const T r = bc - y;
    T s = 0;
#pragma unroll
    for (int m = 0; m < 8; ++m) s += __shfl(r, m, 8);
    if ((tid & 7) == 0) sbc[c >> 3] = s;
  }
  __syncthreads();
  // coarsest: weighted-Jacobi sweeps from zero (k_coarsest)
  for (int c = tid; c < nc; c += CTPB) xa[c] = omega * sbc[c] / sdc[c];
  __syncthreads();
  T* cur = xa;
  T* nxt = xb;
  for (int s = 1; s < sweeps; ++s) {
    for (int c = tid; c < nc; c += CTPB) {
      T y = sdc[c] * cur[c];
      for (int k = 0; k < Wc; ++k) {
        const int j = scl[k * nc + c];
        if (j < nc) y += sv[k * nc + c] * cur[j];
      }
      nxt[c] = cur[c] + omega * (sbc[c] - y) / sdc[c];
    }
    __syncthreads();
    T* t = cur; cur = nxt; nxt = t;
  }
  // up: y = x0 + sc P xc (aggregate of a padded cell: c >> 3), one post-sweep (k_prolong_smooth)
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int c = q * CTPB + tid;
    if (c >= n) continue;
    const T yc = sx[c] + sc * cur[c >> 3];
    T ay = sD[c] * yc;
#pragma unroll
    for (int k = 0; k < TAIL_W; ++k) {
      if (k >= W) break;
      const int j = cj[q][k];
      if (j < n) ay += cv[q][k] * (sx[j] + sc * cur[j >> 3]);
    }
    const T bc = sb[c];
    xo[c] = yc + omega * (bc - ay) / sD[c];
  }
}

// ---------------------------------------------------------------- agglomerated coarsest level (Amg::global)
// rank's packed rows (nmax rows of wg values + the diagonal): local coarsest couplings (slots < wloc of the
// level's own ELL; up to wc), the external couplings summed in double from the level-0 halo coefficients
// in their listed order (slots wc .. wc + we), the diagonal; padding rows (I >= nloc) are a unit diagonal
template <class T>
__global__ void k_gc_pack(int nmax, int nloc, int wloc, int wc, int we, const T* __restrict__ valc,
                          const T* __restrict__ Dc, const double* __restrict__ val0, const int* __restrict__ estart,
                          const int* __restrict__ esrc, double* __restrict__ send) {
  const int I = blockIdx.x * blockDim.x + threadIdx.x;
  if (I >= nmax) return;
  const int wg = wc + we;
  double* o = send + (long)I * (wg + 1);
  for (int k = 0; k < wc; ++k) o[k] = (I < nloc && k < wloc) ? (double)valc[(long)k * nloc + I] : 0.0;
  for (int e = 0; e < we; ++e) {
    double s = 0.0;
    for (int q = estart[I * we + e]; q < estart[I * we + e + 1]; ++q) s += val0[esrc[q]];
    o[wc + e] = s;
  }
  o[wg] = I < nloc ? (double)Dc[I] : 1.0;
}
// every rank unpacks the gathered rows identically: global row G = r nmax + I
template <class T>
__global__ void k_gc_unpack(int ng, int nmax, int wg, const double* __restrict__ recv, T* __restrict__ val,
                            T* __restrict__ D) {
  const int G = blockIdx.x * blockDim.x + threadIdx.x;
  if (G >= ng) return;
  const double* s = recv + (long)(G / nmax) * nmax * (wg + 1) + (long)(G % nmax) * (wg + 1);
  for (int k = 0; k < wg; ++k) val[(long)k * ng + G] = (T)s[k];
  D[G] = (T)s[wg];
}
template <class T>
__global__ void k_gc_bpack(int nmax, int nloc, const T* __restrict__ b, double* __restrict__ out) {
  const int I = blockIdx.x * blockDim.x + threadIdx.x;
  if (I < nmax) out[I] = I < nloc ? (double)b[I] : 0.0;
}

// ---------------------------------------------------------------- host: hierarchy
// (aggregation in amg_graph.h, shared with the CPU-A baseline; here the result is uploaded)
void build_next(AmgLevel& f, const std::vector<int>& fcol, const Graph& g, AmgLevel& c, std::vector<int>& ccol,
                Graph& cg, hipStream_t st, int passes, std::vector<int>& agg_host) {
  AmgCoarse k = amg_coarsen(fcol, f.W, f.n, g, passes);
  agg_host = k.agg;
  f.agg.upload(k.agg, st);
  f.mstart.upload(k.mstart, st);
  f.members.upload(k.members, st);
  f.gstart.upload(k.gstart, st);
  f.gsrc.upload(k.gsrc, st);
  c.n = k.nc;
  c.W = k.Wc;
  ccol.swap(k.ccol);
  cg = std::move(k.cg);
  c.col.upload(ccol, st);
}


// Levels 1 .. L-2 renumbered so that the (at most 8) members of every aggregate sit in one aligned group
// of 8 consecutive cells: level l's cell of parent J, sibling m (members in their previous order) gets
// index 8 J' + m, J' the parent's new index (numbered the same way from the coarsest level down). Unused
// slots are empty cells (no couplings, unit diagonal, zero right-hand side). The restriction of such a
// level is then a sum over 8 adjacent lanes inside the smoothing kernel (k_smooth_res_r8), so levels
// 1 .. L-2 need one launch on the way down instead of two. Level 0 keeps the mesh order. Member order
// inside an aggregate is unchanged, so every restriction sums the same values in the same order.
// On return fin_aggs / last_col hold the final fine -> coarse maps and the coarsest level's columns (they
// are left untouched when the levels stay plain).
void pad_levels(Ctx& x, const std::vector<int>& col0, const std::vector<std::vector<int>>& aggs,
                std::vector<std::vector<int>>& fin_aggs, std::vector<int>& last_col) {
  Amg& a = x.amg;
  const int L = (int)a.lv.size();
  if (L < 3) return;
  // new index of every level-l cell, from the coarsest level down (level L-1 keeps its numbering)
  std::vector<std::vector<int>> pi(L);
  std::vector<int> nn(L);
  nn[L - 1] = a.lv[L - 1].n;
  pi[L - 1].resize(nn[L - 1]);
  std::iota(pi[L - 1].begin(), pi[L - 1].end(), 0);
  for (int l = L - 2; l >= 1; --l) {
    const std::vector<int>& ag = aggs[l];   // level l -> level l + 1 (old numbering)
    std::vector<int> cnt(a.lv[l + 1].n, 0);
    pi[l].resize(a.lv[l].n);
    for (int v = 0; v < a.lv[l].n; ++v) {
      const int m = cnt[ag[v]]++;
      if (m >= 8) return;                    // an aggregate of more than 8 cells: keep the plain levels
      pi[l][v] = 8 * pi[l + 1][ag[v]] + m;
    }
    nn[l] = 8 * nn[l + 1];
  }
  // rebuild the member lists, coarse columns and Galerkin lists in the new numbering
  std::vector<int> fcol = col0;
  int Wf = a.lv[0].W, nf = a.lv[0].n;
  for (int l = 0; l + 1 < L; ++l) {
    AmgCoarse r;
    r.agg.resize(nf);
    if (l == 0) for (int v = 0; v < nf; ++v) r.agg[v] = pi[1][aggs[0][v]];
    else for (int v = 0; v < nf; ++v) r.agg[v] = v >> 3;
    amg_level_data(fcol, Wf, nf, nn[l + 1], r);
    AmgLevel& f = a.lv[l];
    AmgLevel& c = a.lv[l + 1];
    f.agg.upload(r.agg, x.stream);
    f.mstart.upload(r.mstart, x.stream);
    f.members.upload(r.members, x.stream);
    f.gstart.upload(r.gstart, x.stream);
    f.gsrc.upload(r.gsrc, x.stream);
    c.n = r.nc;
    c.W = r.Wc;
    c.col.upload(r.ccol, x.stream);
    fcol.swap(r.ccol);
    fin_aggs[l] = r.agg;
    Wf = c.W;
    nf = c.n;
  }
  last_col = fcol;
  DFMI_HIP(hipStreamSynchronize(x.stream));
  a.padded = true;
}

// Amg::global (amg.h): the agglomerated coarsest level. Collective: every rank calls it in its first
// pressure solve. col0: level-0 ELL columns [W][C] (>= C: halo entries); aggs: fine -> coarse maps of the
// final levels; lcol: the local coarsest level's columns.
void global_setup(Ctx& x, const std::vector<int>& col0, const std::vector<std::vector<int>>& aggs,
                  const std::vector<int>& lcol) {
  Amg& a = x.amg;
  a.global = false;
  const int L = (int)a.lv.size();
  const int C = x.C, W0 = x.ell.W, H = x.H, R = x.nranks;
  const int nloc = a.lv[L - 1].n, wloc = a.lv[L - 1].W;
  // collective size agreement: (levels, coarsest cells, coarsest width) of every rank
  auto gather = [&](const std::vector<double>& mine) {
    const long n = (long)mine.size();
    DevBuf<double> sb, rb;
    sb.upload(mine, x.stream);
    rb.alloc((size_t)n * R);
    halo_allgather(x, sb.p, rb.p, n);
    std::vector<double> all((size_t)n * R);
    DFMI_HIP(hipMemcpyAsync(all.data(), rb.p, all.size() * sizeof(double), hipMemcpyDeviceToHost, x.stream));
    DFMI_HIP(hipStreamSynchronize(x.stream));
    return all;
  };
  int nmax = 0, wc = 0, we = 0;
  {
    const std::vector<double> all = gather({(double)L, (double)nloc, (double)wloc});
    for (int r = 0; r < R; ++r) {
      if (all[3 * r] < 2) return;   // a rank without coarse levels: block-Jacobi everywhere
      nmax = std::max(nmax, (int)all[3 * r + 1]); wc = std::max(wc, (int)all[3 * r + 2]);
    }
  }
  // coarsest-level aggregate of every fine cell, and of the cell across every processor face
  std::vector<int> cid(C);
  for (int c = 0; c < C; ++c) {
    int v = c;
    for (int l = 0; l + 1 < L; ++l) v = aggs[l][v];
    cid[c] = v;
  }
  std::vector<double> ids((size_t)C + H, -1.0);
  for (int c = 0; c < C; ++c) ids[c] = cid[c];
  DevBuf<double> dids;
  dids.upload(ids, x.stream);
  HaloItem it{dids.p, dids.p, 1, (long)C + H, (long)C + H, false};
  halo_update(x, &it, 1);
  DFMI_HIP(hipMemcpyAsync(ids.data(), dids.p, ids.size() * sizeof(double), hipMemcpyDeviceToHost, x.stream));
  DFMI_HIP(hipStreamSynchronize(x.stream));
  std::vector<int> hpeer(H, -1);
  for (int p = 0; p < x.P; ++p) {
    if (x.pkind[p] != 2) continue;
    for (int i = 0; i < x.psize[p]; ++i) {
      const int h = x.h_hidx[x.poff[p] + i];
      if (h >= 0) hpeer[h] = x.peer[p];
    }
  }
  // external couplings of each local coarsest row: (peer, peer's coarsest id) -> level-0 ELL sources k C + c
  // (a rank-local inconsistency is agreed on in the next all-gather, so every rank throws together instead of
  // the others blocking in a collective the failed rank never joins)
  std::vector<std::map<std::pair<int, int>, std::vector<int>>> ext(nloc);
  bool bad = false;
  for (int c = 0; c < C; ++c)
    for (int k = 0; k < W0; ++k) {
      const int j = col0[(size_t)k * C + c];
      if (j < C) continue;
      const int h = j - C;
      if (!(hpeer[h] >= 0 && ids[j] >= 0)) { bad = true; continue; }
      ext[cid[c]][{hpeer[h], (int)ids[j]}].push_back(k * C + c);
    }
  int wext = 0;
  for (auto& e : ext) wext = std::max(wext, (int)e.size());
  {
    const std::vector<double> all = gather({(double)wext, bad ? 1.0 : 0.0});
    bool any_bad = false;
    for (int r = 0; r < R; ++r) { we = std::max(we, (int)all[2 * r]); any_bad = any_bad || all[2 * r + 1] != 0.0; }
    DFMI_CHECK(!any_bad, "AMG: processor face without a peer aggregate (on some rank)");
  }
  const int ng = R * nmax, wg = wc + we;
  if (ng > COARSEST || (size_t)ng * wg > LDS_ENT) return;   // the same decision on every rank
  // external sum lists per (row, slot), ordered by global column
  std::vector<int> es(1, 0), esrc;
  std::vector<double> pc((size_t)nmax * wg);
  const int G0 = x.rank * nmax;
  for (int I = 0; I < nmax; ++I) {
    for (int k = 0; k < wc; ++k) pc[(size_t)I * wg + k] = G0 + ((I < nloc && k < wloc) ? lcol[(size_t)k * nloc + I] : I);
    int e = 0;
    if (I < nloc)
      for (auto& kv : ext[I]) {   // (peer, id) ascending = global column ascending
        pc[(size_t)I * wg + wc + e] = kv.first.first * nmax + kv.first.second;
        for (int q : kv.second) esrc.push_back(q);
        es.push_back((int)esrc.size());
        ++e;
      }
    for (; e < we; ++e) { pc[(size_t)I * wg + wc + e] = G0 + I; es.push_back((int)esrc.size()); }
  }
  if (esrc.empty()) esrc.push_back(0);
  const std::vector<double> allc = gather(pc);
  std::vector<int> gcol((size_t)wg * ng);
  for (int G = 0; G < ng; ++G)
    for (int k = 0; k < wg; ++k) gcol[(size_t)k * ng + G] = (int)allc[(size_t)G * wg + k];
  a.g_col.upload(gcol, x.stream);
  a.e_start.upload(es, x.stream);
  a.e_src.upload(esrc, x.stream);
  a.g_send.alloc((size_t)nmax * (wg + 1));
  a.g_recv.alloc((size_t)ng * (wg + 1));
  a.g_bs.alloc(nmax);
  a.g_bg.alloc(ng);
  if (a.fp32) { a.g_fval.alloc((size_t)wg * ng); a.g_fD.alloc(ng); a.g_fx.alloc(ng); }
  else { a.g_val.alloc((size_t)wg * ng); a.g_D.alloc(ng); a.g_x.alloc(ng); }
  DFMI_HIP(hipStreamSynchronize(x.stream));
  a.nmax = nmax; a.ng = ng; a.wc = wc; a.we = we; a.wg = wg; a.nloc = nloc;
  a.global = true;
}

}  // namespace

void amg_setup(Ctx& x) {
  Amg& a = x.amg;
  a.lv.clear();
  a.omega = x.opt("amg.omega");
  a.coarse_sweeps = (int)x.opt("amg.coarsest_sweeps");
  a.l0_sweeps = std::max(1, (int)x.opt("amg.presweeps"));
  a.coarsest = std::min(COARSEST, std::max(8, (int)x.opt("amg.coarsest_size")));
  a.overcorr = x.opt("amg.overcorrection");
  a.fp32 = x.opt("amg.precision") != 64;
  const int C = x.C;
  // level 0: the solver ELL (columns >= C are halo entries, dropped in the preconditioner)
  std::vector<int> col((size_t)x.ell.W * C);
  DFMI_HIP(hipMemcpy(col.data(), x.ell.col.p, col.size() * sizeof(int), hipMemcpyDeviceToHost));
  // geometric strength |Sf| * deltaCoeffs per coupling (faces and cyclic slots)
  std::vector<double> mag(x.Fs), dcf(x.Fs), bmag(x.B), bdc(x.B);   // face storage order
  if (x.Fs) {
    DFMI_HIP(hipMemcpy(mag.data(), x.magSf.p, x.Fs * sizeof(double), hipMemcpyDeviceToHost));
    DFMI_HIP(hipMemcpy(dcf.data(), x.dc.p, x.Fs * sizeof(double), hipMemcpyDeviceToHost));
  }
  if (x.B) {
    DFMI_HIP(hipMemcpy(bmag.data(), x.bmagSf.p, x.B * sizeof(double), hipMemcpyDeviceToHost));
    DFMI_HIP(hipMemcpy(bdc.data(), x.bdc.p, x.B * sizeof(double), hipMemcpyDeviceToHost));
  }
  std::vector<int> fo(x.F), fn(x.F);
  std::vector<double> fs(x.F);
  for (int f = 0; f < x.F; ++f) { fo[f] = x.h_own[f]; fn[f] = x.h_nei[f]; fs[f] = mag[x.h_fst[f]] * dcf[x.h_fst[f]]; }
  std::vector<int> co, cn;
  std::vector<double> cs;
  for (int p = 0; p < x.P; ++p) {
    if (x.pkind[p] != 1) continue;
    const int q = x.cyc_nbr[p];
    for (int i = 0; i < x.psize[p]; ++i) {
      const int b = x.poff[p] + i;
      co.push_back(x.h_bfc[b]); cn.push_back(x.h_bfc[x.poff[q] + i]); cs.push_back(bmag[b] * bdc[b]);
    }
  }
  Graph g = strength_graph(C, fo, fn, fs, co, cn, cs);
  a.lv.emplace_back();
  a.lv[0].n = C;
  a.lv[0].W = x.ell.W;
  std::vector<int> fcol = col;
  std::vector<std::vector<int>> aggs;   // host copies of each level's fine -> coarse map
  // several ranks: the rank-local levels stop at coarsest / nranks cells, below them the agglomerated level
  const bool want_global = x.nranks > 1 && halo_active(x) && x.on("amg.global_coarse");
  const int cap = want_global ? std::max(8, a.coarsest / x.nranks) : a.coarsest;
  auto too_big = [&](const AmgLevel& l) { return l.n > cap || (size_t)l.n * l.W > 6144; };
  while (too_big(a.lv.back())) {
    AmgLevel c;
    std::vector<int> ccol;
    Graph cg;
    aggs.emplace_back();
    build_next(a.lv.back(), fcol, g, c, ccol, cg, x.stream, (int)x.opt(a.lv.size() == 1 ? "amg.pairwise_passes_l0" : "amg.pairwise_passes"),
               aggs.back());
    DFMI_HIP(hipStreamSynchronize(x.stream));
    const bool stalled = c.n * 2 > a.lv.back().n;
    a.lv.push_back(std::move(c));
    fcol.swap(ccol);
    g = std::move(cg);
    if (stalled) break;
  }
  DFMI_CHECK(!too_big(a.lv.back()) || a.lv.back().n <= 8, "AMG coarsening stalled above the coarsest-level capacity");
  a.padded = false;
  a.global = false;
  std::vector<std::vector<int>> fin_aggs = aggs;
  std::vector<int> last_col = fcol;
  if (x.on("amg.padded")) pad_levels(x, col, aggs, fin_aggs, last_col);
  if (a.lv.size() == 1) a.fp32 = false;   // a single level writes z directly: keep it in double
  for (size_t l = 0; l < a.lv.size(); ++l) {
    AmgLevel& v = a.lv[l];
    const size_t nv = v.n, ne = (size_t)v.W * v.n;
    if (a.fp32) {
      v.fval.alloc(ne); v.fD.alloc(nv);
      if (l > 0) v.fb.alloc(nv);
      v.fx.alloc(nv); v.fr.alloc(nv); v.fxo.alloc(nv);
      if (l == 0 && a.l0_sweeps > 1) v.fr2.alloc(nv);
    } else {
      if (l > 0) { v.val.alloc(ne); v.D.alloc(nv); v.b.alloc(nv); }
      v.x.alloc(nv); v.r.alloc(nv); v.xo.alloc(nv);
      if (l == 0 && a.l0_sweeps > 1) v.r2.alloc(nv);
    }
    if (l == 0 && a.l0_sweeps > 1) v.zt.alloc(nv);
  }
  if (want_global) global_setup(x, col, fin_aggs, last_col);
  // measured (in-process ranks of 64^3): p-iterations per solve 14 / 17 / 19 -> 12 / 14 / 14-15 for 2 / 4 / 8
  // ranks (one rank: 12) for two more halo exchanges per PCG iteration; amg.halo_l0 = 0: block-Jacobi
  a.halo_l0 = x.nranks > 1 && halo_active(x) && x.on("amg.halo_l0") && a.lv.size() >= 2 && a.l0_sweeps == 1;
  if (a.halo_l0) a.hy.alloc((size_t)C + x.H);
  // the last two levels as one single-workgroup launch (k_vtail; amg.tail = 0: the launch chain)
  {
    const int L = (int)a.lv.size();
    a.tail = x.on("amg.tail") && a.padded && a.fp32 && L >= 3 && a.lv[L - 2].n <= TAIL_N &&
             a.lv[L - 2].n % 8 == 0 && a.lv[L - 2].W <= TAIL_W && a.lv[L - 1].n <= COARSEST &&
             (size_t)a.lv[L - 1].n * a.lv[L - 1].W <= LDS_ENT && !a.global;
  }
  a.ready = true;
}

// Per solve: coarse operators from the level-0 values (val0 [W][C], D0 = diag + internalCoeffs).
void amg_galerkin(Ctx& x, const double* val0, const double* D0) {
  Amg& a = x.amg;
  if (a.fp32) {   // the level-0 smoother reads a single-precision copy of the solver's ELL operator
    AmgLevel& l0 = a.lv[0];
    KScope _ks(x, "k_round_f32");
    if (a.face) {   // ... or of the face and slot coefficients the face-wise level 0 reads
      const long nf = 3L * a.dfo.C, nb = std::max(x.B, 1);
      if (a.fup.n < (size_t)nf) a.fup.alloc(nf);
      if (a.fbc.n < (size_t)nb) a.fbc.alloc(nb);
      hipLaunchKernelGGL(k_round_f32, dim3(2048), dim3(TPB), 0, x.stream, nf, a.dfo.up, a.fup.p);
      if (x.B) hipLaunchKernelGGL(k_round_f32, dim3(256), dim3(TPB), 0, x.stream, (long)x.B, a.dfo.bc, a.fbc.p);
      a.ffo = FaceOp<float>{1, a.dfo.nx, a.dfo.ny, a.dfo.nz, a.dfo.C, a.fup.p, a.fbc.p, a.dfo.csStart, a.dfo.csSlot,
                            a.dfo.scol};
    } else {
      hipLaunchKernelGGL(k_round_f32, dim3(2048), dim3(TPB), 0, x.stream, (long)l0.W * l0.n, val0, l0.fval.p);
    }
    hipLaunchKernelGGL(k_round_f32, dim3(512), dim3(TPB), 0, x.stream, (long)l0.n, D0, l0.fD.p);
    DFMI_HIP(hipGetLastError());
  }
  for (size_t l = 0; l + 1 < a.lv.size(); ++l) {
    AmgLevel& f = a.lv[l];
    AmgLevel& c = a.lv[l + 1];
    KScope _ks(x, "k_galerkin");
    const dim3 g(blocks_for((long)c.n * (c.W + 1), TPB));
    if (!a.fp32)
      hipLaunchKernelGGL((k_galerkin<double, double>), g, dim3(TPB), 0, x.stream, c.n, c.W + 1, f.gstart.p, f.gsrc.p,
                         l == 0 ? val0 : (const double*)f.val.p, l == 0 ? D0 : (const double*)f.D.p, c.val.p, c.D.p);
    else if (l == 0)   // coarse sums from the fp64 fine values, rounded once
      hipLaunchKernelGGL((k_galerkin<double, float>), g, dim3(TPB), 0, x.stream, c.n, c.W + 1, f.gstart.p, f.gsrc.p,
                         val0, D0, c.fval.p, c.fD.p);
    else
      hipLaunchKernelGGL((k_galerkin<float, float>), g, dim3(TPB), 0, x.stream, c.n, c.W + 1, f.gstart.p, f.gsrc.p,
                         (const float*)f.fval.p, (const float*)f.fD.p, c.fval.p, c.fD.p);
    DFMI_HIP(hipGetLastError());
  }
  if (a.global) {   // the agglomerated level: pack this rank's rows, all-gather, unpack (identical on every rank)
    AmgLevel& c = a.lv.back();
    KScope _ks(x, "k_gc_pack");
    const dim3 gp(blocks_for(a.nmax, TPB)), gu(blocks_for(a.ng, TPB));
    if (a.fp32)
      hipLaunchKernelGGL(k_gc_pack<float>, gp, dim3(TPB), 0, x.stream, a.nmax, a.nloc, c.W, a.wc, a.we,
                         (const float*)c.fval.p, (const float*)c.fD.p, val0, a.e_start.p, a.e_src.p, a.g_send.p);
    else
      hipLaunchKernelGGL(k_gc_pack<double>, gp, dim3(TPB), 0, x.stream, a.nmax, a.nloc, c.W, a.wc, a.we,
                         (const double*)c.val.p, (const double*)c.D.p, val0, a.e_start.p, a.e_src.p, a.g_send.p);
    DFMI_HIP(hipGetLastError());
    halo_allgather(x, a.g_send.p, a.g_recv.p, (long)a.nmax * (a.wg + 1));
    if (a.fp32)
      hipLaunchKernelGGL(k_gc_unpack<float>, gu, dim3(TPB), 0, x.stream, a.ng, a.nmax, a.wg, (const double*)a.g_recv.p,
                         a.g_fval.p, a.g_fD.p);
    else
      hipLaunchKernelGGL(k_gc_unpack<double>, gu, dim3(TPB), 0, x.stream, a.ng, a.nmax, a.wg, (const double*)a.g_recv.p,
                         a.g_val.p, a.g_D.p);
    DFMI_HIP(hipGetLastError());
  }
}

namespace {

template <class K0, class K6, class... A>
void launch_w(int W, dim3 g, hipStream_t st, K0 k0, K6 k6, A... a) {
  if (W == 6) hipLaunchKernelGGL(k6, g, dim3(TPB), 0, st, a...);
  else hipLaunchKernelGGL(k0, g, dim3(TPB), 0, st, a...);
}

// z = M^-1 r in precision T; block partials of r.z (one per block of the level-0 grid) into `partial`
template <class T>
void apply_t(Ctx& x, const double* val0, const double* D0, ColView col0, const double* r, double* z,
             double* partial, int nblk, const double* act, bool l0_done, const CgStop& stop) {
  constexpr bool F = std::is_same<T, float>::value;
  Amg& a = x.amg;
  const int L = (int)a.lv.size();
  const T om = (T)a.omega, sc = (T)a.overcorr;
  auto VAL = [&](int l) -> const T* {
    if constexpr (F) return a.lv[l].fval.p; else return l == 0 ? val0 : (const double*)a.lv[l].val.p;
  };
  auto DD = [&](int l) -> const T* {
    if constexpr (F) return a.lv[l].fD.p; else return l == 0 ? D0 : (const double*)a.lv[l].D.p;
  };
  // level 0: the solver rows (row classes where built); coarse levels: explicit columns
  auto COL = [&](int l) { return l == 0 ? col0 : ColView{a.lv[l].col.p, nullptr, nullptr, a.lv[l].W}; };
  auto FO = [&]() -> FaceOp<T> { if constexpr (F) return a.ffo; else return a.dfo; };
  auto RAW = [&](int l) { return l == 0 ? col0.col : (const int*)a.lv[l].col.p; };
  auto BV = [&](int l) -> T* { if constexpr (F) return a.lv[l].fb.p; else return a.lv[l].b.p; };
  auto XV = [&](int l) -> T* { if constexpr (F) return a.lv[l].fx.p; else return a.lv[l].x.p; };
  auto RV = [&](int l) -> T* { if constexpr (F) return a.lv[l].fr.p; else return a.lv[l].r.p; };
  auto XO = [&](int l) -> T* { if constexpr (F) return a.lv[l].fxo.p; else return a.lv[l].xo.p; };
  // the last two levels in one workgroup (k_vtail): the down loop stops above level L - 2
  const bool tail = F && a.tail;
  const int ldown = tail ? L - 2 : L - 1;
  // down: smooth from zero + residual, restrict (folding the level-0 restriction into level 1's launch, each level-1
  // thread summing its own and its six neighbours' member residuals, measured 14.6 -> 15.1-15.3 ms per step, round 5)
  for (int l = 0; l < ldown; ++l) {
    AmgLevel& f = a.lv[l];
    const dim3 g(blocks_for(f.n, TPB));
    if (l > 0 && a.padded) {   // aggregates in aligned groups of 8: smoothing and restriction in one launch
      KScope _ks(x, "k_smooth_res");
      launch_w(f.W, g, x.stream, k_smooth_res_r8<0, T>, k_smooth_res_r8<6, T>, f.n, f.W, RAW(l), VAL(l), DD(l),
               (const T*)BV(l), om, XV(l), BV(l + 1), act);
      continue;
    }
    T* rcur = RV(l);
    if (!(l == 0 && l0_done)) {
      KScope _ks(x, "k_smooth_res");
      if (l == 0 && a.halo_l0)   // r and the diagonal carry the exchanged halo entries (solve_pcg)
        launch_w(f.W, g, x.stream, k_smooth_res_h<0, T>, k_smooth_res_h<6, T>, f.n, f.W, COL(0), VAL(0), DD(0), r,
                 a.dS_full, om, XV(0), RV(0), act);
      else if (l == 0 && a.face)
        hipLaunchKernelGGL((k_smooth_res<0, T, double, true>), g, dim3(TPB), 0, x.stream, f.n, f.W, COL(0), VAL(0),
                           DD(0), r, om, XV(0), RV(0), act, FO());
      else if (l == 0)
        launch_w(f.W, g, x.stream, k_smooth_res<0, T, double>, k_smooth_res<6, T, double>, f.n, f.W, COL(0), VAL(0),
                 DD(0), r, om, XV(0), RV(0), act, FaceOp<T>{});
      else
        launch_w(f.W, g, x.stream, k_smooth_res<0, T, T>, k_smooth_res<6, T, T>, f.n, f.W, COL(l), VAL(l), DD(l),
                 (const T*)BV(l), om, XV(l), RV(l), act, FaceOp<T>{});
    }
    if (l == 0 && a.l0_sweeps > 1) {   // further pre-sweeps, the residual carried along
      T* ralt;
      if constexpr (F) ralt = f.fr2.p; else ralt = f.r2.p;
      for (int s = 1; s < a.l0_sweeps; ++s) {
        KScope _ks(x, "k_smooth_step");
        launch_w(f.W, g, x.stream, k_smooth_step<0, T>, k_smooth_step<6, T>, f.n, f.W, COL(0), VAL(0), DD(0),
                 (const T*)rcur, om, XV(0), ralt, act);
        std::swap(rcur, ralt);
      }
    }
    {
      KScope _ks(x, "k_restrict");
      hipLaunchKernelGGL(k_restrict<T>, dim3(blocks_for(a.lv[l + 1].n, TPB)), dim3(TPB), 0, x.stream, a.lv[l + 1].n,
                         f.mstart.p, f.members.p, (const T*)rcur, BV(l + 1), act,
                         l == 0 && l0_done ? stop : CgStop{});
    }
  }
  // coarsest: the agglomerated level (every rank's coarsest right-hand sides gathered, the global level
  // smoothed redundantly), or this rank's own coarsest level
  T* gx = nullptr;
  if constexpr (F) gx = a.g_fx.p; else gx = a.g_x.p;
  if (tail) {
    AmgLevel& f = a.lv[L - 2];
    AmgLevel& c = a.lv[L - 1];
    KScope _ks(x, "k_vtail");
    if constexpr (!F) DFMI_CHECK(false, "k_vtail: fp32 V-cycle only");
    else if (f.W == 6)
      hipLaunchKernelGGL((k_vtail<6, T>), dim3(1), dim3(CTPB), 0, x.stream, f.n, f.W, RAW(L - 2), VAL(L - 2), DD(L - 2),
                         (const T*)BV(L - 2), c.n, c.W, RAW(L - 1), VAL(L - 1), DD(L - 1), om, sc, a.coarse_sweeps,
                         XO(L - 2), act);
    else
      hipLaunchKernelGGL((k_vtail<0, T>), dim3(1), dim3(CTPB), 0, x.stream, f.n, f.W, RAW(L - 2), VAL(L - 2), DD(L - 2),
                         (const T*)BV(L - 2), c.n, c.W, RAW(L - 1), VAL(L - 1), DD(L - 1), om, sc, a.coarse_sweeps,
                         XO(L - 2), act);
    // the corrected iterate of level L - 2 feeds the next finer prolongation (as after k_prolong_smooth)
    if constexpr (F) std::swap(f.fx, f.fxo); else std::swap(f.x, f.xo);
  } else if (a.global && L > 1) {
    KScope _ks(x, "k_coarsest");
    hipLaunchKernelGGL(k_gc_bpack<T>, dim3(blocks_for(a.nmax, TPB)), dim3(TPB), 0, x.stream, a.nmax, a.nloc,
                       (const T*)BV(L - 1), a.g_bs.p);
    DFMI_HIP(hipGetLastError());
    halo_allgather(x, a.g_bs.p, a.g_bg.p, a.nmax);
    const T* gv;
    const T* gd;
    if constexpr (F) { gv = a.g_fval.p; gd = a.g_fD.p; } else { gv = a.g_val.p; gd = a.g_D.p; }
    hipLaunchKernelGGL((k_coarsest<T, double, T>), dim3(1), dim3(CTPB), 0, x.stream, a.ng, a.wg, (const int*)a.g_col.p,
                       gv, gd, (const double*)a.g_bg.p, om, a.coarse_sweeps, gx, act);
  } else {
    AmgLevel& c = a.lv[L - 1];
    KScope _ks(x, "k_coarsest");
    if (L > 1)
      hipLaunchKernelGGL((k_coarsest<T, T, T>), dim3(1), dim3(CTPB), 0, x.stream, c.n, c.W, RAW(L - 1), VAL(L - 1),
                         DD(L - 1), (const T*)BV(L - 1), om, a.coarse_sweeps, XV(L - 1), act);
    else if constexpr (!F)   // single level (double only): solve straight into z
      hipLaunchKernelGGL((k_coarsest<double, double, double>), dim3(1), dim3(CTPB), 0, x.stream, c.n, c.W, col0.col, val0,
                         D0, r, om, a.coarse_sweeps, z, act);
  }
  // the coarse correction the level above the coarsest prolongates: this rank's rows of the global solution
  auto XC = [&](int l) -> const T* { return (a.global && l + 1 == L - 1) ? gx + (long)x.rank * a.nmax : XV(l + 1); };
  if (L == 1) {
    KScope _ks(x, "k_dot_partial");
    hipLaunchKernelGGL(k_dot_partial, dim3(nblk), dim3(TPB), 0, x.stream, x.C, r, (const double*)z, partial);
  }
  // up: prolongate the coarse correction + one smoothing sweep
  for (int l = tail ? L - 3 : L - 2; l >= 0; --l) {
    AmgLevel& f = a.lv[l];
    KScope _ks(x, "k_prolong_smooth");
    if (l == 0 && a.halo_l0) {   // prolongate, exchange the iterate, post-sweep with the processor columns
      hipLaunchKernelGGL(k_prolong_y<T>, dim3(blocks_for(f.n, TPB)), dim3(TPB), 0, x.stream, f.n, (const T*)XV(0),
                         (const int*)f.agg.p, XC(0), sc, a.hy.p, act);
      DFMI_HIP(hipGetLastError());
      HaloItem it{a.hy.p, a.hy.p, 1, (long)f.n + x.H, (long)f.n + x.H, false};
      halo_update(x, &it, 1);
      launch_w(f.W, dim3(nblk), x.stream, k_post_smooth_h<0, T>, k_post_smooth_h<6, T>, f.n, f.W, COL(0), VAL(0), DD(0),
               r, (const double*)a.hy.p, om, z, partial, act);
    } else if (l == 0 && a.face) {   // one post-sweep (face mode needs l0_sweeps == 1)
      hipLaunchKernelGGL((k_prolong_smooth<0, T, double, double, true>), dim3(nblk), dim3(TPB), 0, x.stream, f.n, f.W,
                         COL(0), VAL(0), DD(0), r, (const T*)XV(0), (const int*)f.agg.p, XC(0), om, sc, z, partial,
                         act, FO());
    } else if (l == 0) {
      // with ns post-sweeps the outputs alternate zt / z so that the last one lands in z
      const int ns = a.l0_sweeps;
      auto outk = [&](int k) { return ((ns - k) % 2 == 0) ? z : f.zt.p; };   // k = 1 .. ns
      launch_w(f.W, dim3(nblk), x.stream, k_prolong_smooth<0, T, double, double>, k_prolong_smooth<6, T, double, double>,
               f.n, f.W, COL(0), VAL(0), DD(0), r, (const T*)XV(0), (const int*)f.agg.p, XC(0), om, sc,
               outk(1), ns == 1 ? partial : (double*)nullptr, act, FaceOp<T>{});
      for (int k = 2; k <= ns; ++k) {
        KScope _ks2(x, "k_jacobi_sweep");
        launch_w(f.W, dim3(nblk), x.stream, k_jacobi_sweep<0, T, double, double>, k_jacobi_sweep<6, T, double, double>,
                 f.n, f.W, COL(0), VAL(0), DD(0), r, (const double*)outk(k - 1), om, outk(k),
                 k == ns ? partial : (double*)nullptr, act);
      }
    } else {
      launch_w(f.W, dim3(blocks_for(f.n, TPB)), x.stream, k_prolong_smooth<0, T, T, T>, k_prolong_smooth<6, T, T, T>,
               f.n, f.W, COL(l), VAL(l), DD(l), (const T*)BV(l), (const T*)XV(l), (const int*)f.agg.p,
               XC(l), om, sc, XO(l), (double*)nullptr, act, FaceOp<T>{});
      // the corrected x of this level feeds the next finer prolongation
      if constexpr (F) std::swap(f.fx, f.fxo); else std::swap(f.x, f.xo);
    }
  }
  DFMI_HIP(hipGetLastError());
}

}  // namespace

namespace {
template <class T>
AmgView<T> amg_view_t(Ctx& x, const double* val0, const double* D0, const int* col0) {
  constexpr bool F = std::is_same<T, float>::value;
  Amg& a = x.amg;
  AmgView<T> v;
  v.L = (int)a.lv.size();
  DFMI_CHECK(v.L <= AMG_MAXL, "AMG: too many levels for the single-workgroup V-cycle");
  for (int l = 0; l < v.L; ++l) {
    AmgLevel& g = a.lv[l];
    v.n[l] = g.n; v.W[l] = g.W;
    v.col[l] = l == 0 ? col0 : (const int*)g.col.p;
    if constexpr (F) {
      v.val[l] = g.fval.p; v.D[l] = g.fD.p; v.b[l] = g.fb.p; v.x[l] = g.fx.p; v.r[l] = g.fr.p; v.xo[l] = g.fxo.p;
    } else {
      v.val[l] = l == 0 ? val0 : (const double*)g.val.p; v.D[l] = l == 0 ? D0 : (const double*)g.D.p;
      v.b[l] = g.b.p; v.x[l] = g.x.p; v.r[l] = g.r.p; v.xo[l] = g.xo.p;
    }
    v.agg[l] = g.agg.p; v.mstart[l] = g.mstart.p; v.members[l] = g.members.p;
  }
  v.omega = (T)a.omega; v.sc = (T)a.overcorr; v.sweeps = a.coarse_sweeps;
  return v;
}
}  // namespace

AmgView<float> amg_view_f32(Ctx& x, const int* col0) { return amg_view_t<float>(x, nullptr, nullptr, col0); }
AmgView<double> amg_view_f64(Ctx& x, const double* val0, const double* D0, const int* col0) {
  return amg_view_t<double>(x, val0, D0, col0);
}

bool amg_l0_fusable(const Ctx& x) {
  const Amg& a = x.amg;
  return a.fp32 && a.lv.size() >= 2 && a.l0_sweeps == 1;
}

void amg_apply(Ctx& x, const double* val0, const double* D0, ColView col0, const double* r, double* z,
               double* partial, int nblk, const double* active, bool l0_done, const CgStop& stop) {
  Amg& a = x.amg;
  DFMI_CHECK(!l0_done || amg_l0_fusable(x), "AMG: level-0 sweep fused on an unsupported configuration");
  CommTag _ct(x, x.comm.tag + " amg");
  if (a.fp32) apply_t<float>(x, val0, D0, col0, r, z, partial, nblk, active, l0_done, stop);
  else apply_t<double>(x, val0, D0, col0, r, z, partial, nblk, active, l0_done, stop);
}

}  // namespace dfmi
