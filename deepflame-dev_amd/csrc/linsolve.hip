// linsolve.hip -- Krylov solvers on LDU storage (replaces the AmgX path, reference
// src_gpu/AmgXSolver.cu:184-340 and dfMatrixDataBase.cu:166-177, and the per-matrix
// ldu_to_csr gathers dfMatrixOpBase.cu:2276-2352 / dfUEqn.cu:836-894).
//
// The SpMV gathers directly from lower/upper/diag plus the coupled boundary coefficients (cyclic
// partner cells, processor halo values), so no 20 B x nnz CSR copy is made per matrix. Systems that
// share the sparsity pattern are solved as one batch (grid.y = system): the 3 U components, and all
// non-inert species of the Y equation (their matrices are independent, so the reference's sequential
// species loop is a batch here). Preconditioner: Jacobi on diag + internalCoeffs. Convergence: AmgX
// RELATIVE_INI L2 (||r|| <= tol ||r0||), per system. All reductions are two-stage and fixed-order,
// hence deterministic. Scalars live on the device; the host reads only the per-system residual and
// active flag every `check` iterations (inactive systems turn every kernel into a no-op).
#include "dfmi_ctx.h"
#include <cmath>

namespace dfmi {
namespace {

constexpr int TPB = 256;
constexpr int NW = TPB / 64;

struct Sys {
  int nsys;
  const double *lower, *upper, *diag, *source, *ic, *bc;
  long lstride, ustride, dstride, sstride, bstride;
  double* x; long xstride;
  const double* xhalo;   // processor neighbour values of x, [nsys][B] (may be null)
};

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  return v;
}
// block-reduce NV values into partial[(s*nblk + blk)*NV + k]
template <int NV> __device__ __forceinline__ void block_partials(double (&v)[NV], double* partial, int s, int nblk) {
  __shared__ double red[NW][NV];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) { const double r = wave_sum(v[k]); if (lane == 0) red[wid][k] = r; }
  __syncthreads();
  if (threadIdx.x < NV) {
    double a = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) a += red[w][threadIdx.x];
    partial[((long)s * nblk + blockIdx.x) * NV + threadIdx.x] = a;
  }
}
// fixed-order sum of the block partials of system s (one block per system)
template <int NV> __device__ __forceinline__ void finalize_sums(const double* partial, int s, int nblk, double (&out)[NV]) {
  __shared__ double red[NW][NV];
  double v[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = 0.0;
  for (int i = threadIdx.x; i < nblk; i += TPB)
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] += partial[((long)s * nblk + i) * NV + k];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) { const double r = wave_sum(v[k]); if (lane == 0) red[wid][k] = r; }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    double a = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) a += red[w][k];
    out[k] = a;
  }
}

// y = A x for system s: diag + internalCoeffs on the diagonal, lower/upper off-diagonal, and
// -boundaryCoeffs * x_neighbour across coupled slots (lduMatrix::Amul + updateMatrixInterfaces)
__device__ __forceinline__ double amul(const MeshView& m, const int8_t* ty, const Sys& q, int s, const double* dS,
                                       const double* xv, int c) {
  const double* L = q.lower + s * q.lstride;
  const double* U = q.upper + s * q.ustride;
  const double* bc = q.bc + s * q.bstride;
  double y = dS[c] * xv[c];
  const int e1 = m.nbrStart[c + 1];
  for (int k = m.nbrStart[c]; k < e1; ++k) { const int f = m.nbrFace[k]; y += L[f] * xv[m.own[f]]; }
  const int e2 = m.ownStart[c + 1];
  for (int f = m.ownStart[c]; f < e2; ++f) y += U[f] * xv[m.nei[f]];
  const int e3 = m.cbStart[c + 1];
  for (int k = m.cbStart[c]; k < e3; ++k) {
    const int b = m.cbSlot[k];
    const int t = ty[b];
    if (!bc_coupled(t)) continue;
    const int pc = m.partner[b];
    const double xn = pc >= 0 ? xv[pc] : q.xhalo[(long)s * m.B + b];
    y -= bc[b] * xn;
  }
  return y;
}

// dS = diag + sum internalCoeffs (fvMatrix::addBoundaryDiag), rhs = source + non-coupled boundaryCoeffs
// (fvMatrix::addBoundarySource(source, false)), in slot order
__global__ void k_setup(MeshView m, const int8_t* ty, Sys q, double* dS, double* rhs, const int* sys_map) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const int s = blockIdx.y;
  if (c >= m.C) return;
  const int ms = sys_map ? sys_map[s] : s;
  const double* ic = q.ic + ms * q.bstride;
  const double* bc = q.bc + ms * q.bstride;
  double d = q.diag[ms * q.dstride + c];
  double r = q.source[ms * q.sstride + c];
  const int e3 = m.cbStart[c + 1];
  for (int k = m.cbStart[c]; k < e3; ++k) {
    const int b = m.cbSlot[k];
    const int t = ty[b];
    if (t == EMPTY) continue;
    d += ic[b];
  }
  for (int k = m.cbStart[c]; k < e3; ++k) {
    const int b = m.cbSlot[k];
    const int t = ty[b];
    if (t == EMPTY || bc_coupled(t)) continue;
    r += bc[b];
  }
  dS[(long)s * m.C + c] = d;
  rhs[(long)s * m.C + c] = r;
}

// ---- BiCGStab kernels. State per system (scal[s*8+k]): 0 rho, 1 rho_old, 2 alpha, 3 omega,
// 4 res0, 5 res, 6 active, 7 iters.
__global__ void k_bcg_init(MeshView m, const int8_t* ty, Sys q, const int* sys_map, const double* dS, const double* rhs,
                           double* r, double* r0, double* p, double* v, double* partial, int nblk) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const int s = blockIdx.y;
  const long C = m.C;
  double acc[2] = {0.0, 0.0};
  if (c < m.C) {
    const int ms = sys_map ? sys_map[s] : s;
    const double* xv = q.x + ms * q.xstride;
    const double ax = amul(m, ty, q, ms, dS + s * C, xv, c);
    const double rr = rhs[s * C + c] - ax;
    r[s * C + c] = rr; r0[s * C + c] = rr; p[s * C + c] = 0.0; v[s * C + c] = 0.0;
    acc[0] = rr * rr;
    acc[1] = rr * rr;
  }
  block_partials<2>(acc, partial, s, nblk);
}
__global__ void k_bcg_init_fin(double* partial, int nblk, double* scal, double tol, double abs_tol) {
  const int s = blockIdx.x;
  double v[2];
  finalize_sums<2>(partial, s, nblk, v);
  if (threadIdx.x == 0) {
    double* st = scal + s * 8;
    const double res = sqrt(v[0]);
    st[0] = v[1]; st[1] = 1.0; st[2] = 1.0; st[3] = 1.0; st[4] = res; st[5] = res; st[7] = 0;
    st[6] = (res > abs_tol && res > 0.0) ? 1.0 : 0.0;
  }
}
// p = r + beta (p - omega v); phat = p / dS; then v = A phat needs a separate pass
__global__ void k_bcg_p(int C, const double* scal, const double* r, double* p, const double* v, const double* dS,
                        double* phat) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const int s = blockIdx.y;
  const double* st = scal + s * 8;
  if (c >= C || st[6] == 0.0) return;
  const long i = (long)s * C + c;
  const double beta = (st[0] / st[1]) * (st[2] / st[3]);
  const double pv = r[i] + beta * (p[i] - st[3] * v[i]);
  p[i] = pv;
  phat[i] = pv / dS[i];
}
// out = A in, plus partial dots: (r0, out) [NV=1] or (out, sv), (out, out) [NV=2]
template <int NV>
__global__ void k_bcg_spmv(MeshView m, const int8_t* ty, Sys q, const int* sys_map, const double* scal,
                           const double* dS, const double* in, double* out, const double* dotv, double* partial,
                           int nblk) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const int s = blockIdx.y;
  const long C = m.C;
  double acc[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) acc[k] = 0.0;
  if (scal[s * 8 + 6] == 0.0) return;   // uniform per block
  if (c < m.C) {
    const int ms = sys_map ? sys_map[s] : s;
    const double y = amul(m, ty, q, ms, dS + s * C, in + s * C, c);
    out[s * C + c] = y;
    if (NV == 1) acc[0] = dotv[s * C + c] * y;
    else { acc[0] = y * dotv[s * C + c]; if (NV > 1) acc[NV - 1] = y * y; }
  }
  block_partials<NV>(acc, partial, s, nblk);
}
__global__ void k_bcg_alpha(double* partial, int nblk, double* scal) {
  const int s = blockIdx.x;
  if (scal[s * 8 + 6] == 0.0) return;
  double v[1];
  finalize_sums<1>(partial, s, nblk, v);
  if (threadIdx.x == 0) {
    double* st = scal + s * 8;
    if (v[0] == 0.0) { st[6] = 0.0; return; }
    st[2] = st[0] / v[0];
  }
}
// s = r - alpha v; shat = s / dS
__global__ void k_bcg_s(int C, const double* scal, const double* r, const double* v, const double* dS, double* sv,
                        double* shat) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const int s = blockIdx.y;
  const double* st = scal + s * 8;
  if (c >= C || st[6] == 0.0) return;
  const long i = (long)s * C + c;
  const double ss = r[i] - st[2] * v[i];
  sv[i] = ss;
  shat[i] = ss / dS[i];
}
__global__ void k_bcg_omega(double* partial, int nblk, double* scal) {
  const int s = blockIdx.x;
  if (scal[s * 8 + 6] == 0.0) return;
  double v[2];
  finalize_sums<2>(partial, s, nblk, v);
  if (threadIdx.x == 0) {
    double* st = scal + s * 8;
    st[3] = v[1] != 0.0 ? v[0] / v[1] : 0.0;
  }
}
// x += alpha phat + omega shat; r = s - omega t; partials (r,r), (r0,r)
__global__ void k_bcg_x(int C, Sys q, const int* sys_map, const double* scal, const double* phat, const double* shat,
                        const double* sv, const double* t, double* r, const double* r0, double* partial, int nblk) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const int s = blockIdx.y;
  const double* st = scal + s * 8;
  if (st[6] == 0.0) return;
  double acc[2] = {0.0, 0.0};
  if (c < C) {
    const long i = (long)s * C + c;
    const int ms = sys_map ? sys_map[s] : s;
    double* xv = q.x + ms * q.xstride;
    xv[c] = xv[c] + st[2] * phat[i] + st[3] * shat[i];
    const double rr = sv[i] - st[3] * t[i];
    r[i] = rr;
    acc[0] = rr * rr;
    acc[1] = r0[i] * rr;
  }
  block_partials<2>(acc, partial, s, nblk);
}
__global__ void k_bcg_fin(double* partial, int nblk, double* scal, double tol, double abs_tol, int max_iter) {
  const int s = blockIdx.x;
  if (scal[s * 8 + 6] == 0.0) return;
  double v[2];
  finalize_sums<2>(partial, s, nblk, v);
  if (threadIdx.x == 0) {
    double* st = scal + s * 8;
    const double res = sqrt(v[0]);
    st[5] = res;
    st[7] += 1.0;
    st[1] = st[0];
    st[0] = v[1];
    if (res <= tol * st[4] || res <= abs_tol || st[7] >= max_iter || st[0] == 0.0 || st[3] == 0.0) st[6] = 0.0;
  }
}

// ---- PCG (Jacobi) for the symmetric pressure matrix. scal: 0 rz, 1 alpha, 2 beta, 4 res0, 5 res, 6 active, 7 iters
__global__ void k_cg_init(MeshView m, const int8_t* ty, Sys q, const double* dS, const double* rhs, double* r, double* z,
                          double* p, double* partial, int nblk) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  double acc[2] = {0.0, 0.0};
  if (c < m.C) {
    const double ax = amul(m, ty, q, 0, dS, q.x, c);
    const double rr = rhs[c] - ax;
    const double zz = rr / dS[c];
    r[c] = rr; z[c] = zz; p[c] = zz;
    acc[0] = rr * zz; acc[1] = rr * rr;
  }
  block_partials<2>(acc, partial, 0, nblk);
}
__global__ void k_cg_init_fin(double* partial, int nblk, double* scal, double abs_tol) {
  double v[2];
  finalize_sums<2>(partial, 0, nblk, v);
  if (threadIdx.x == 0) {
    const double res = sqrt(v[1]);
    scal[0] = v[0]; scal[4] = res; scal[5] = res; scal[7] = 0;
    scal[6] = (res > abs_tol && res > 0.0) ? 1.0 : 0.0;
  }
}
__global__ void k_cg_spmv(MeshView m, const int8_t* ty, Sys q, const double* scal, const double* dS, const double* p,
                          double* qv, double* partial, int nblk) {
  if (scal[6] == 0.0) return;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  double acc[1] = {0.0};
  if (c < m.C) {
    const double y = amul(m, ty, q, 0, dS, p, c);
    qv[c] = y;
    acc[0] = p[c] * y;
  }
  block_partials<1>(acc, partial, 0, nblk);
}
__global__ void k_cg_alpha(double* partial, int nblk, double* scal) {
  if (scal[6] == 0.0) return;
  double v[1];
  finalize_sums<1>(partial, 0, nblk, v);
  if (threadIdx.x == 0) { if (v[0] == 0.0) { scal[6] = 0.0; return; } scal[1] = scal[0] / v[0]; }
}
__global__ void k_cg_x(int C, double* x, const double* scal, const double* p, const double* qv, double* r, double* z,
                       const double* dS, double* partial, int nblk) {
  if (scal[6] == 0.0) return;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  double acc[2] = {0.0, 0.0};
  if (c < C) {
    const double a = scal[1];
    x[c] = x[c] + a * p[c];
    const double rr = r[c] - a * qv[c];
    r[c] = rr;
    const double zz = rr / dS[c];
    z[c] = zz;
    acc[0] = rr * zz; acc[1] = rr * rr;
  }
  block_partials<2>(acc, partial, 0, nblk);
}
__global__ void k_cg_fin(double* partial, int nblk, double* scal, double tol, double abs_tol, int max_iter) {
  if (scal[6] == 0.0) return;
  double v[2];
  finalize_sums<2>(partial, 0, nblk, v);
  if (threadIdx.x == 0) {
    const double res = sqrt(v[1]);
    scal[5] = res;
    scal[7] += 1.0;
    scal[2] = scal[0] != 0.0 ? v[0] / scal[0] : 0.0;
    scal[0] = v[0];
    if (res <= tol * scal[4] || res <= abs_tol || scal[7] >= max_iter) scal[6] = 0.0;
  }
}
__global__ void k_cg_p(int C, const double* scal, const double* z, double* p) {
  if (scal[6] == 0.0) return;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  p[c] = z[c] + scal[2] * p[c];
}

struct Workspace {
  DevBuf<double> buf;
  DevBuf<double> scal;
  DevBuf<int> sysmap;
  std::vector<double> hscal;
};
Workspace& ws(Ctx& x) {
  static std::map<Ctx*, Workspace> w;
  return w[&x];
}

}  // namespace

SolveStats solve_bicgstab(Ctx& x, const char* eqn, int nsys, const int* sys_map_host, const double* lower, long lstride,
                          const double* upper, long ustride, const double* diag, long dstride, const double* source,
                          long sstride, const double* ic, const double* bc, long bstride, const char* type_field,
                          double* xsol, long xstride, const SolverCfg& cfg) {
  const long C = x.C;
  const int nblk = blocks_for(C, TPB);
  Workspace& W = ws(x);
  const size_t need = (size_t)nsys * C * 10 + (size_t)nsys * nblk * 2 + 64;
  if (W.buf.n < need) W.buf.alloc(need);
  if (W.scal.n < (size_t)nsys * 8) W.scal.alloc(nsys * 8);
  const int* smap = nullptr;
  if (sys_map_host) {
    W.sysmap.upload(sys_map_host, nsys, x.stream);
    smap = W.sysmap.p;
  }
  const long N = nsys * C;
  double *dS = W.buf.p, *rhs = dS + N, *r = rhs + N, *r0 = r + N, *p = r0 + N, *v = p + N, *phat = v + N,
         *sv = phat + N, *shat = sv + N, *t = shat + N, *partial = t + N;
  Sys q{nsys, lower, upper, diag, source, ic, bc, lstride, ustride, dstride, sstride, bstride, xsol, xstride,
        x.fields.count("halo_x") ? x.f("halo_x") : nullptr};
  MeshView m = x.view();
  const int8_t* ty = x.st(type_field);
  dim3 g(nblk, nsys), bl(TPB);
  { KScope _ks(x, "k_setup"); hipLaunchKernelGGL(k_setup, g, bl, 0, x.stream, m, ty, q, dS, rhs, smap); }
  { KScope _ks(x, "k_bcg_init"); hipLaunchKernelGGL(k_bcg_init, g, bl, 0, x.stream, m, ty, q, smap, dS, rhs, r, r0, p, v, partial, nblk); }
  { KScope _ks(x, "k_bcg_init_fin"); hipLaunchKernelGGL(k_bcg_init_fin, dim3(nsys), bl, 0, x.stream, partial, nblk, W.scal.p, cfg.tol, cfg.abs_tol); }
  DFMI_HIP(hipGetLastError());
  W.hscal.resize(nsys * 8);
  int it = 0;
  const int check = 2;
  bool synced = false;
  while (it < cfg.max_iter) {
    for (int k = 0; k < check && it < cfg.max_iter; ++k, ++it) {
      { KScope _ks(x, "k_bcg_p"); hipLaunchKernelGGL(k_bcg_p, g, bl, 0, x.stream, (int)C, W.scal.p, r, p, v, dS, phat); }
      { KScope _ks(x, "k_bcg_spmv"); hipLaunchKernelGGL(k_bcg_spmv<1>, g, bl, 0, x.stream, m, ty, q, smap, W.scal.p, dS, phat, v, r0, partial, nblk); }
      { KScope _ks(x, "k_bcg_alpha"); hipLaunchKernelGGL(k_bcg_alpha, dim3(nsys), bl, 0, x.stream, partial, nblk, W.scal.p); }
      { KScope _ks(x, "k_bcg_s"); hipLaunchKernelGGL(k_bcg_s, g, bl, 0, x.stream, (int)C, W.scal.p, r, v, dS, sv, shat); }
      { KScope _ks(x, "k_bcg_spmv"); hipLaunchKernelGGL(k_bcg_spmv<2>, g, bl, 0, x.stream, m, ty, q, smap, W.scal.p, dS, shat, t, sv, partial, nblk); }
      { KScope _ks(x, "k_bcg_omega"); hipLaunchKernelGGL(k_bcg_omega, dim3(nsys), bl, 0, x.stream, partial, nblk, W.scal.p); }
      { KScope _ks(x, "k_bcg_x"); hipLaunchKernelGGL(k_bcg_x, g, bl, 0, x.stream, (int)C, q, smap, W.scal.p, phat, shat, sv, t, r, r0, partial, nblk); }
      { KScope _ks(x, "k_bcg_fin"); hipLaunchKernelGGL(k_bcg_fin, dim3(nsys), bl, 0, x.stream, partial, nblk, W.scal.p, cfg.tol, cfg.abs_tol, cfg.max_iter); }
    }
    DFMI_HIP(hipGetLastError());
    DFMI_HIP(hipMemcpyAsync(W.hscal.data(), W.scal.p, nsys * 8 * sizeof(double), hipMemcpyDeviceToHost, x.stream));
    DFMI_HIP(hipStreamSynchronize(x.stream));
    synced = true;
    bool any = false;
    for (int s = 0; s < nsys; ++s) any |= W.hscal[s * 8 + 6] != 0.0;
    if (!any) break;
  }
  if (!synced) {
    DFMI_HIP(hipMemcpyAsync(W.hscal.data(), W.scal.p, nsys * 8 * sizeof(double), hipMemcpyDeviceToHost, x.stream));
    DFMI_HIP(hipStreamSynchronize(x.stream));
  }
  SolveStats st;
  for (int s = 0; s < nsys; ++s) {
    st.iters = std::max(st.iters, (int)W.hscal[s * 8 + 7]);
    st.res0 = std::max(st.res0, W.hscal[s * 8 + 4]);
    st.res = std::max(st.res, W.hscal[s * 8 + 4] > 0 ? W.hscal[s * 8 + 5] / W.hscal[s * 8 + 4] : 0.0);
  }
  x.last_stats[eqn] = st;
  return st;
}

SolveStats solve_pcg(Ctx& x, const char* eqn, const double* lower, const double* upper, const double* diag,
                     const double* source, const double* ic, const double* bc, const char* type_field, double* xsol,
                     double* bxsol, const SolverCfg& cfg) {
  (void)bxsol;
  const long C = x.C;
  const int nblk = blocks_for(C, TPB);
  Workspace& W = ws(x);
  const size_t need = (size_t)C * 6 + (size_t)nblk * 2 + 64;
  if (W.buf.n < need) W.buf.alloc(need);
  if (W.scal.n < 8) W.scal.alloc(8);
  double *dS = W.buf.p, *rhs = dS + C, *r = rhs + C, *z = r + C, *p = z + C, *qv = p + C, *partial = qv + C;
  Sys q{1, lower, upper, diag, source, ic, bc, 0, 0, 0, 0, 0, xsol, 0, x.fields.count("halo_x") ? x.f("halo_x") : nullptr};
  MeshView m = x.view();
  const int8_t* ty = x.st(type_field);
  dim3 g(nblk), bl(TPB);
  { KScope _ks(x, "k_setup"); hipLaunchKernelGGL(k_setup, dim3(nblk, 1), bl, 0, x.stream, m, ty, q, dS, rhs, (const int*)nullptr); }
  { KScope _ks(x, "k_cg_init"); hipLaunchKernelGGL(k_cg_init, g, bl, 0, x.stream, m, ty, q, dS, rhs, r, z, p, partial, nblk); }
  { KScope _ks(x, "k_cg_init_fin"); hipLaunchKernelGGL(k_cg_init_fin, dim3(1), bl, 0, x.stream, partial, nblk, W.scal.p, cfg.abs_tol); }
  DFMI_HIP(hipGetLastError());
  W.hscal.resize(8);
  int it = 0;
  const int check = 8;
  while (it < cfg.max_iter) {
    for (int k = 0; k < check && it < cfg.max_iter; ++k, ++it) {
      { KScope _ks(x, "k_cg_spmv"); hipLaunchKernelGGL(k_cg_spmv, g, bl, 0, x.stream, m, ty, q, W.scal.p, dS, p, qv, partial, nblk); }
      { KScope _ks(x, "k_cg_alpha"); hipLaunchKernelGGL(k_cg_alpha, dim3(1), bl, 0, x.stream, partial, nblk, W.scal.p); }
      { KScope _ks(x, "k_cg_x"); hipLaunchKernelGGL(k_cg_x, g, bl, 0, x.stream, (int)C, xsol, W.scal.p, p, qv, r, z, dS, partial, nblk); }
      { KScope _ks(x, "k_cg_fin"); hipLaunchKernelGGL(k_cg_fin, dim3(1), bl, 0, x.stream, partial, nblk, W.scal.p, cfg.tol, cfg.abs_tol, cfg.max_iter); }
      { KScope _ks(x, "k_cg_p"); hipLaunchKernelGGL(k_cg_p, g, bl, 0, x.stream, (int)C, W.scal.p, z, p); }
    }
    DFMI_HIP(hipGetLastError());
    DFMI_HIP(hipMemcpyAsync(W.hscal.data(), W.scal.p, 8 * sizeof(double), hipMemcpyDeviceToHost, x.stream));
    DFMI_HIP(hipStreamSynchronize(x.stream));
    if (W.hscal[6] == 0.0) break;
  }
  SolveStats st;
  st.iters = (int)W.hscal[7];
  st.res0 = W.hscal[4];
  st.res = W.hscal[4] > 0 ? W.hscal[5] / W.hscal[4] : 0.0;
  x.last_stats[eqn] = st;
  return st;
}

}  // namespace dfmi
