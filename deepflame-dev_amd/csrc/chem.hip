// chem.hip -- per-cell stiff chemistry on MI355X.
//
// Semantics of the reference chemistry step (dfChemistryModel::solveSingle,
// src/dfChemistryModel/dfChemistryModel.C:737-780; GPU ABI precedent opencc_ode_all, YEqn.H:45-77):
// every cell is a closed constant-volume reactor at FIXED temperature and density integrated over
// the flow time step; the species source is RR_i = (Y_i(dt) - Y_i(0)) rho / dt. Kinetics follow
// Cantera GasKinetics: Arrhenius rates, three-body efficiencies, Lindemann/Troe fall-off, reverse
// rates from NASA7 equilibrium constants.
//
// Integrator: ROS3 Rosenbrock (L-stable, order 3, embedded order-2 error estimate, one Jacobian and
// one LU per step) with adaptive step size; alternative (option chem.method = 1): linearly-implicit
// Euler extrapolation with step sequence 1, 2, 3. Analytic Jacobian: mass action, third-body factors and
// the fall-off rate constants' [M]-dependence (without the latter the stiff 1D-flame cells needed 2-5x
// more steps: a Rosenbrock method loses order with an inexact Jacobian). Tolerances mirror the reference's CVODE settings (relTol 1e-6, absTol 1e-10 on
// mass fractions) by default.
//
// Scheduling: cells are launched in descending order of the integrator steps they needed in the
// previous solve (counting sort, k_bin_*): a wave costs its slowest lane, and on the reference TGV
// state natural order loads waves at 23% (mean / per-wave max); binned, k_chem drops 7.3 -> 1.9 ms.
//
// Layout: one cell per lane, 64-lane workgroups. Per-lane rate constants (they depend only on T,
// which is frozen) and the per-lane S x S iteration matrix live in LDS as [entry][lane]
// (bank-conflict free); state vectors live in registers (compile-time S). The mechanism arrays are
// wave-uniform (scalar loads).
#include "dfmi_ctx.h"
#include <cmath>
#include <cstdlib>

namespace dfmi {
namespace {

constexpr int LANES = 64;
constexpr double RU = 8314.46261815324;
constexpr double P_ATM = 101325.0;

struct ChemMech {
  int R, ndd;
  const int* idata;    // [R][8]: type, reversible, n_reac, n_prod, has_T2
  const int* irs;      // [R][6]: reactant ids (3), product ids (3), -1 padded
  const double* dd;    // [R][ndd]: A b Ta nu_r[3] nu_p[3] A0 b0 Ta0 troe[4] eff[S]
  const double* nasa;  // [S][15]
  const double* W;     // [S]
};

template <int S> struct Lane {
  double* kf;   // LDS [R][LANES]
  double* k0;
  double* ikc;  // 1/Kc, 0 for irreversible
  double* A;    // LDS [S*S][LANES]
  int lane;
  __device__ double& K(double* b, int r) const { return b[r * LANES + lane]; }
  __device__ double& M(int i, int j) const { return A[(i * S + j) * LANES + lane]; }
};

template <int S>
__device__ void rate_constants(const ChemMech& m, const Lane<S>& L, double T) {
  const double lnT = log(T), rT = 1.0 / T;
  double g[S];
#pragma unroll
  for (int i = 0; i < S; ++i) {   // g_i / RT from NASA7
    const double* row = m.nasa + i * 15;
    const double* a = T > row[0] ? row + 1 : row + 8;
    const double h = a[0] + a[1] * T / 2 + a[2] * T * T / 3 + a[3] * T * T * T / 4 + a[4] * T * T * T * T / 5 + a[5] / T;
    const double s = a[0] * lnT + a[1] * T + a[2] * T * T / 2 + a[3] * T * T * T / 3 + a[4] * T * T * T * T / 4 + a[6];
    g[i] = h - s;
  }
  for (int r = 0; r < m.R; ++r) {
    const int* id = m.idata + r * 8;
    const int* ix = m.irs + r * 6;
    const double* d = m.dd + (long)r * m.ndd;
    L.K(L.kf, r) = d[0] * exp(d[1] * lnT - d[2] * rT);
    L.K(L.k0, r) = id[0] >= 2 ? d[9] * exp(d[10] * lnT - d[11] * rT) : 0.0;
    double ik = 0.0;
    if (id[1]) {
      double dG = 0.0, dnu = 0.0;
      for (int k = 0; k < 3; ++k) {
        const int ip = ix[3 + k], ir = ix[k];
#pragma unroll
        for (int i = 0; i < S; ++i) {   // wave-uniform species ids; unrolled select keeps g in registers
          if (ip == i) { dG += d[6 + k] * g[i]; }
          if (ir == i) { dG -= d[3 + k] * g[i]; }
        }
        if (ip >= 0) dnu += d[6 + k];
        if (ir >= 0) dnu -= d[3 + k];
      }
      // 1/Kc = exp(dG) (p_atm / RT)^-dnu
      ik = exp(dG - dnu * log(P_ATM / (RU * T)));
    }
    L.K(L.ikc, r) = ik;
  }
}

template <int S> __device__ __forceinline__ double sel(const double (&v)[S], int i) {
  double o = 0.0;
#pragma unroll
  for (int k = 0; k < S; ++k) o = (k == i) ? v[k] : o;
  return o;
}
template <int S> __device__ __forceinline__ void add_at(double (&v)[S], int i, double a) {
#pragma unroll
  for (int k = 0; k < S; ++k) if (k == i) v[k] += a;
}

// effective rate coefficient and the third-body factor of reaction r
template <int S>
__device__ __forceinline__ void rcoef(const ChemMech& m, const Lane<S>& L, int r, double T, const double (&C)[S],
                                      double& k, double& Mf, double& Mc) {
  const int* id = m.idata + r * 8;
  const double* d = m.dd + (long)r * m.ndd;
  k = L.K(L.kf, r);
  Mf = 1.0;
  Mc = 0.0;
  if (id[0] == 0) return;
  double M = 0.0;
#pragma unroll
  for (int i = 0; i < S; ++i) M += d[17 + i] * C[i];
  if (id[0] == 1) { Mf = M; Mc = 1.0; return; }
  const double Pr = L.K(L.k0, r) * M / k;
  double F = 1.0;
  if (id[0] == 3) {
    const double a = d[12], T3 = d[13], T1 = d[14], T2 = d[15];
    const double Fc = (1 - a) * exp(-T / T3) + a * exp(-T / T1) + (id[4] ? exp(-T2 / T) : 0.0);
    const double lFc = log10(fmax(Fc, 1e-300));
    const double c = -0.4 - 0.67 * lFc, n = 0.75 - 1.27 * lFc;
    const double lPr = log10(fmax(Pr, 1e-300));
    const double f1 = (lPr + c) / (n - 0.14 * (lPr + c));
    F = exp10(lFc / (1 + f1 * f1));
  }
  k = k * Pr / (1 + Pr) * F;
}

// d fo / d[M] of a fall-off reaction (k = k_inf fo, fo = Pr / (1 + Pr) F): the [M]-dependence of the rate
// constant, which Rosenbrock methods need in the Jacobian for their order (chem_codegen.py derives the
// same expression for the generated kernels)
template <int S>
__device__ __forceinline__ double falloff_dfo(const ChemMech& m, const Lane<S>& L, int r, double T, const double (&C)[S]) {
  const int* id = m.idata + r * 8;
  const double* d = m.dd + (long)r * m.ndd;
  double M = 0.0;
#pragma unroll
  for (int i = 0; i < S; ++i) M += d[17 + i] * C[i];
  const double kinf = L.K(L.kf, r), k0 = L.K(L.k0, r);
  const double Pr = k0 * M / kinf;
  double F = 1.0, corr = 0.0;
  if (id[0] == 3) {
    const double a = d[12], T3 = d[13], T1 = d[14], T2 = d[15];
    const double Fc = (1 - a) * exp(-T / T3) + a * exp(-T / T1) + (id[4] ? exp(-T2 / T) : 0.0);
    const double lFc = log10(fmax(Fc, 1e-300));
    const double c = -0.4 - 0.67 * lFc, n = 0.75 - 1.27 * lFc;
    const double lPr = log10(fmax(Pr, 1e-300));
    const double u = n - 0.14 * (lPr + c);
    const double f1 = (lPr + c) / u;
    F = exp10(lFc / (1 + f1 * f1));
    corr = F * 2.0 * lFc * f1 * n / ((1.0 + Pr) * (1.0 + f1 * f1) * (1.0 + f1 * f1) * u * u);
  }
  return k0 / kinf * (F / ((1.0 + Pr) * (1.0 + Pr)) - corr);
}

__device__ __forceinline__ double ipow(double c, double nu) {
  return nu == 1.0 ? c : (nu == 2.0 ? c * c : (nu == 3.0 ? c * c * c : pow(c, nu)));
}
__device__ __forceinline__ double dipow(double c, double nu) {   // d/dc c^nu
  return nu == 1.0 ? 1.0 : (nu == 2.0 ? 2.0 * c : (nu == 3.0 ? 3.0 * c * c : nu * pow(c, nu - 1.0)));
}

// w = dC/dt
template <int S>
__device__ void rhs(const ChemMech& m, const Lane<S>& L, double T, const double (&C)[S], double (&w)[S]) {
#pragma unroll
  for (int i = 0; i < S; ++i) w[i] = 0.0;
  for (int r = 0; r < m.R; ++r) {
    const int* id = m.idata + r * 8;
    const int* ix = m.irs + r * 6;
    const double* d = m.dd + (long)r * m.ndd;
    double k, Mf, Mc;
    rcoef<S>(m, L, r, T, C, k, Mf, Mc);
    double f = k, b = id[1] ? k * L.K(L.ikc, r) : 0.0;
    for (int j = 0; j < 3; ++j) {
      if (ix[j] >= 0) f *= ipow(sel<S>(C, ix[j]), d[3 + j]);
      if (ix[3 + j] >= 0) b *= ipow(sel<S>(C, ix[3 + j]), d[6 + j]);
    }
    const double q = Mf * (f - b);
    for (int j = 0; j < 3; ++j) {
      if (ix[j] >= 0) add_at<S>(w, ix[j], -d[3 + j] * q);
      if (ix[3 + j] >= 0) add_at<S>(w, ix[3 + j], d[6 + j] * q);
    }
  }
}

// A = I - h J  (J = d(dC/dt)/dC, mass-action part + third-body factor)
template <int S>
__device__ void build_matrix(const ChemMech& m, const Lane<S>& L, double T, const double (&C)[S], double h) {
#pragma unroll
  for (int i = 0; i < S; ++i)
#pragma unroll
    for (int j = 0; j < S; ++j) L.M(i, j) = (i == j) ? 1.0 : 0.0;
  for (int r = 0; r < m.R; ++r) {
    const int* id = m.idata + r * 8;
    const int* ix = m.irs + r * 6;
    const double* d = m.dd + (long)r * m.ndd;
    double k, Mf, Mc;
    rcoef<S>(m, L, r, T, C, k, Mf, Mc);
    const double kb = id[1] ? k * L.K(L.ikc, r) : 0.0;
    double cr[3], cp[3];
    for (int j = 0; j < 3; ++j) {
      cr[j] = ix[j] >= 0 ? sel<S>(C, ix[j]) : 1.0;
      cp[j] = ix[3 + j] >= 0 ? sel<S>(C, ix[3 + j]) : 1.0;
    }
    // dq/dC for each participating species (3 reactant slots, 3 product slots)
    double dq[6];
    int sp[6];
    for (int a = 0; a < 3; ++a) {
      double t = k;
      for (int j = 0; j < 3; ++j) if (ix[j] >= 0) t *= (j == a) ? dipow(cr[j], d[3 + j]) : ipow(cr[j], d[3 + j]);
      dq[a] = ix[a] >= 0 ? Mf * t : 0.0;
      sp[a] = ix[a];
      double u = kb;
      for (int j = 0; j < 3; ++j) if (ix[3 + j] >= 0) u *= (j == a) ? dipow(cp[j], d[6 + j]) : ipow(cp[j], d[6 + j]);
      dq[3 + a] = ix[3 + a] >= 0 ? -Mf * u : 0.0;
      sp[3 + a] = ix[3 + a];
    }
    double q0 = 0.0;
    if (Mc != 0.0) {
      double f = k, b = kb;
      for (int j = 0; j < 3; ++j) {
        if (ix[j] >= 0) f *= ipow(cr[j], d[3 + j]);
        if (ix[3 + j] >= 0) b *= ipow(cp[j], d[6 + j]);
      }
      q0 = f - b;
    }
    double qf = 0.0;   // fall-off: (d fo / d[M]) (k_inf prod_f - k_inf / Kc prod_b)
    if (id[0] >= 2) {
      const double kinf = L.K(L.kf, r);
      double f = kinf, b = id[1] ? kinf * L.K(L.ikc, r) : 0.0;
      for (int j = 0; j < 3; ++j) {
        if (ix[j] >= 0) f *= ipow(cr[j], d[3 + j]);
        if (ix[3 + j] >= 0) b *= ipow(cp[j], d[6 + j]);
      }
      qf = falloff_dfo<S>(m, L, r, T, C) * (f - b);
    }
    // rows touched: reactants (-nu_r) and products (+nu_p)
    for (int a = 0; a < 6; ++a) {
      const int row = ix[a];   // reactant slots 0..2, product slots 3..5
      if (row < 0) continue;
      const double nu = a < 3 ? -d[3 + a] : d[6 + (a - 3)];
      for (int bb = 0; bb < 6; ++bb)
        if (sp[bb] >= 0 && dq[bb] != 0.0) L.M(row, sp[bb]) -= h * nu * dq[bb];
      if (Mc != 0.0)
#pragma unroll
        for (int j = 0; j < S; ++j) L.M(row, j) -= h * nu * d[17 + j] * q0;
      if (qf != 0.0)
#pragma unroll
        for (int j = 0; j < S; ++j) L.M(row, j) -= h * nu * d[17 + j] * qf;
    }
  }
}

// in-place LU without pivoting (A = I - hJ is an M-matrix-like perturbation of I); false if singular
template <int S> __device__ bool lu(const Lane<S>& L) {
#pragma unroll
  for (int k = 0; k < S; ++k) {
    const double p = L.M(k, k);
    if (!(fabs(p) > 1e-300)) return false;
    const double ip = 1.0 / p;
#pragma unroll
    for (int i = k + 1; i < S; ++i) {
      const double f = L.M(i, k) * ip;
      L.M(i, k) = f;
#pragma unroll
      for (int j = k + 1; j < S; ++j) L.M(i, j) -= f * L.M(k, j);
    }
  }
  return true;
}
template <int S> __device__ void lu_solve(const Lane<S>& L, double (&b)[S]) {
#pragma unroll
  for (int i = 1; i < S; ++i)
#pragma unroll
    for (int j = 0; j < i; ++j) b[i] -= L.M(i, j) * b[j];
#pragma unroll
  for (int i = S - 1; i >= 0; --i) {
#pragma unroll
    for (int j = i + 1; j < S; ++j) b[i] -= L.M(i, j) * b[j];
    b[i] = b[i] / L.M(i, i);
  }
}

// n_sub linearly-implicit Euler substeps of size h/n_sub from y0 (f0 = rhs(y0) given)
template <int S>
__device__ bool lie(const ChemMech& m, const Lane<S>& L, double T, const double (&y0)[S], const double (&f0)[S],
                    double h, int n_sub, double (&out)[S]) {
  const double hs = h / n_sub;
  build_matrix<S>(m, L, T, y0, hs);
  if (!lu<S>(L)) return false;
  double y[S], f[S];
#pragma unroll
  for (int i = 0; i < S; ++i) { y[i] = y0[i]; f[i] = f0[i]; }
  for (int s = 0; s < n_sub; ++s) {
    if (s > 0) rhs<S>(m, L, T, y, f);
    double dlt[S];
#pragma unroll
    for (int i = 0; i < S; ++i) dlt[i] = hs * f[i];
    lu_solve<S>(L, dlt);
#pragma unroll
    for (int i = 0; i < S; ++i) y[i] += dlt[i];
  }
#pragma unroll
  for (int i = 0; i < S; ++i) out[i] = y[i];
  return true;
}

// One ROS3 step (Sandu et al. 1997, L-stable, order 3 with embedded order 2; the coefficients
// of KPP's Rosenbrock ROS-3): (I - h g J) K_i = h g [f(y + sum a_ij K_j) + sum (c_ij / h) K_j];
// y_new = y + sum m_i K_i, error = sum e_i K_i. One Jacobian and one LU per step; stage 3 reuses
// f of stage 2 (a31 = a21 = 1, a32 = 0).
template <int S>
__device__ bool ros3(const ChemMech& m, const Lane<S>& L, double T, const double (&y)[S], const double (&f0)[S],
                     double h, double (&ynew)[S], double (&err)[S]) {
  constexpr double g = 0.43586652150845899941601945119356;
  constexpr double c21 = -0.10156171083877702091975600115545e1, c31 = 0.40759956452537699824805835358067e1,
                   c32 = 0.92076794298330791242156818474003e1;
  constexpr double m1 = 1.0, m2 = 0.61697947043828245592553615689730e1, m3 = -0.42772256543218573326238373806514;
  constexpr double e1 = 0.5, e2 = -0.29079558716805469821718236208017e1, e3 = 0.22354069897811569627360909276199;
  const double hg = h * g;
  build_matrix<S>(m, L, T, y, hg);
  if (!lu<S>(L)) return false;
  double k1[S], k2[S], k3[S], y2[S], f2[S];
#pragma unroll
  for (int i = 0; i < S; ++i) k1[i] = hg * f0[i];
  lu_solve<S>(L, k1);
#pragma unroll
  for (int i = 0; i < S; ++i) y2[i] = y[i] + k1[i];
  rhs<S>(m, L, T, y2, f2);
  const double rh = 1.0 / h;
#pragma unroll
  for (int i = 0; i < S; ++i) k2[i] = hg * (f2[i] + c21 * rh * k1[i]);
  lu_solve<S>(L, k2);
#pragma unroll
  for (int i = 0; i < S; ++i) k3[i] = hg * (f2[i] + rh * (c31 * k1[i] + c32 * k2[i]));
  lu_solve<S>(L, k3);
#pragma unroll
  for (int i = 0; i < S; ++i) {
    ynew[i] = y[i] + m1 * k1[i] + m2 * k2[i] + m3 * k3[i];
    err[i] = e1 * k1[i] + e2 * k2[i] + e3 * k3[i];
  }
  return true;
}

// ---- cost binning: a wave runs as long as its slowest lane, so cells are handed to the integrator
// ordered by the integrator steps (accepted + rejected) they took in the previous solve, most
// expensive first. The unit is a group of GRP consecutive cells (costed by its most expensive cell). GRP = 1:
// single cells. Measured (round 5, 2M headline): single-cell binning scatters a bucket's cells over the mesh (PMC
// traffic 1.8 GB per solve, 4.4x the state's 0.42 GB) but keeps every wave's lanes at the same cost (wave
// efficiency 1.0): 1.05 ms; groups of 8 (whole 64-B lines per wave: 0.6 GB, 1.44x) lose that (efficiency 0.61):
// 1.25 ms -- the kernel is bound by its FP64 issue, not by these bytes. Counting sort over NBIN buckets, stable
// inside a bucket (ascending group index). Every cell's integration is independent of its position, so the
// order changes timing only, never results. Default: the sort inside 4096-cell tiles (chem.binning = 2, below):
// traffic 2.06 -> 0.72 GB per solve at wave efficiency 0.977, k_chem 1.029 -> 1.046 ms and the binning
// passes 0.074 -> 0.056 ms (no global scan): the same 1.10 ms per step (profiles/r05_pmc_traffic*.json).
constexpr int NBIN = 32, BCB = 256, BCELLS = 4096, GRP = 1;   // 4096 groups per binning block, 16 passes of 256
__device__ inline int cost_bin(double st, double rj) {
  const int c = (int)(st + rj);
  return NBIN - 1 - (c < 0 ? NBIN - 1 : (c > NBIN - 1 ? NBIN - 1 : c));   // bucket 0 = most expensive
}
// bucket of group g: its most expensive cell (steps + rejects; a failed cell, steps < 0, is most expensive)
__device__ inline int group_bin(long n, const double* __restrict__ stats, long g) {
  int b = NBIN - 1;
  for (long c = g * GRP; c < n && c < (g + 1) * GRP; ++c) b = min(b, cost_bin(stats[c], stats[n + c]));
  return b;
}
// the cell lane t integrates: group perm[t / GRP], its (t % GRP)-th cell (>= n: no cell)
__device__ inline long bin_cell(const int* perm, long t) { return perm ? (long)perm[t / GRP] * GRP + t % GRP : t; }
// chem.binning = 2 (tile-local): the counting sort runs inside each tile of BCELLS groups (one binning block) rather
// than over the whole mesh, so a wave's cells come from one tile; the 64-wave tile runs on one XCD (one L2) and every
// line of the state it reads is fetched once for the tile instead of once per cost bucket. XCD x's k-th workgroup
// (hardware order: workgroup p on XCD p % 8) takes block k % TILE_B of tile (k / TILE_B) * 8 + x -- consecutive tiles
// on different XCDs, so a costly region of the mesh spreads over all eight. The grid is padded to 8 tiles.
constexpr int TILE_B = BCELLS * GRP / LANES;
__device__ inline long chem_thread(int tiled) {
  long b = blockIdx.x;
  if (tiled) { const long x = b % 8, k = b / 8; b = ((k / TILE_B) * 8 + x) * TILE_B + k % TILE_B; }
  return b * LANES + threadIdx.x;
}
// per-block bucket counts, bucket-major [NBIN][nb]
__global__ void __launch_bounds__(BCB) k_bin_count(long n, const double* __restrict__ stats, int nb, int* __restrict__ cnt) {
  const long ng = (n + GRP - 1) / GRP;
  __shared__ int h[NBIN];
  if (threadIdx.x < NBIN) h[threadIdx.x] = 0;
  __syncthreads();
  for (int i = 0; i < BCELLS / BCB; ++i) {
    const long g = (long)blockIdx.x * BCELLS + i * BCB + threadIdx.x;
    if (g < ng) atomicAdd(&h[group_bin(n, stats, g)], 1);
  }
  __syncthreads();
  if (threadIdx.x < NBIN) cnt[(long)threadIdx.x * nb + blockIdx.x] = h[threadIdx.x];
}
// exclusive scan of the bucket-major counts in place (one workgroup, contiguous chunk per thread)
__global__ void __launch_bounds__(1024) k_bin_scan(int total, int* __restrict__ cnt) {
  __shared__ int part[1024];
  const int per = (total + 1023) / 1024, b0 = threadIdx.x * per, b1 = min(b0 + per, total);
  int a = 0;
  for (int i = b0; i < b1; ++i) a += cnt[i];
  part[threadIdx.x] = a;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {   // Hillis-Steele inclusive scan of the 1024 partials
    const int v = threadIdx.x >= d ? part[threadIdx.x - d] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  a = part[threadIdx.x] - a;
  for (int i = b0; i < b1; ++i) { const int v = cnt[i]; cnt[i] = a; a += v; }
}
// chem.binning = 2: exclusive offsets inside each binning block's own range of perm (bucket order, block by block)
__global__ void __launch_bounds__(BCB) k_bin_scan_local(int nb, int* __restrict__ cnt) {
  const int blk = blockIdx.x * blockDim.x + threadIdx.x;
  if (blk >= nb) return;
  int a = blk * BCELLS;
  for (int b = 0; b < NBIN; ++b) { const int v = cnt[(long)b * nb + blk]; cnt[(long)b * nb + blk] = a; a += v; }
}
__global__ void __launch_bounds__(BCB) k_bin_scatter(long n, const double* __restrict__ stats, int nb,
                                                     const int* __restrict__ off, int* __restrict__ perm) {
  const long ng = (n + GRP - 1) / GRP;
  __shared__ int wc[BCB / 64][NBIN];
  __shared__ int base[NBIN];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (threadIdx.x < NBIN) base[threadIdx.x] = off[(long)threadIdx.x * nb + blockIdx.x];
  for (int i = 0; i < BCELLS / BCB; ++i) {
    const long g = (long)blockIdx.x * BCELLS + i * BCB + threadIdx.x;
    const int k = g < ng ? group_bin(n, stats, g) : -1;
    int rank = 0;
    for (int b = 0; b < NBIN; ++b) {
      const unsigned long long m = __ballot(k == b);
      if (k == b) rank = __popcll(m & ((1ull << lane) - 1ull));
      if (lane == 0) wc[w][b] = __popcll(m);
    }
    __syncthreads();
    if (k >= 0) {
      int pos = base[k] + rank;
      for (int v = 0; v < w; ++v) pos += wc[v][k];
      perm[pos] = (int)g;
    }
    __syncthreads();
    if (threadIdx.x < NBIN) {
      int a = 0;
      for (int v = 0; v < BCB / 64; ++v) a += wc[v][threadIdx.x];
      base[threadIdx.x] += a;
    }
  }
}

// Cantera's setState_TPY(T, p, Y) (dfChemistryModel.C:755): mass fractions clipped at 0 and
// normalised (Phase::setMassFractions), density = p * meanW / (R T); returns that density and the
// reactor's initial concentrations C_i = rho Y_i / W_i. The reactor then runs at this density (closed,
// constant volume), while RR is scaled by the thermo density the caller passes (problem.rhoi =
// rho_[celli], :771 and :807).
template <int S, class WT>
__device__ __forceinline__ double reactor_state(double T, double p, const double (&Y0)[S], const WT& W, double (&C)[S]) {
  double ys = 0.0;
#pragma unroll
  for (int i = 0; i < S; ++i) ys += fmax(Y0[i], 0.0);
  const double iys = 1.0 / ys;
  double sw = 0.0;
#pragma unroll
  for (int i = 0; i < S; ++i) sw += fmax(Y0[i], 0.0) * iys / W[i];
  const double rho = p / (sw * RU * T);
#pragma unroll
  for (int i = 0; i < S; ++i) C[i] = rho * (fmax(Y0[i], 0.0) * iys) / W[i];
  return rho;
}

template <int S>
__global__ void __launch_bounds__(LANES) k_chem(long n, const int* __restrict__ perm, ChemMech m,
                                                const double* __restrict__ Tf, const double* __restrict__ pf,
                                                const double* __restrict__ rhof, const double* __restrict__ Yf,
                                                double dt, double rtol, double atol, double Tmin, int max_steps,
                                                int method, double* __restrict__ RR, double* __restrict__ stats,
                                                int* __restrict__ fail, int tiled, const double* __restrict__ hc,
                                                double* __restrict__ Qdot) {
  extern __shared__ double lds[];
  Lane<S> L;
  L.lane = threadIdx.x;
  L.kf = lds;
  L.k0 = lds + (long)m.R * LANES;
  L.ikc = lds + 2L * m.R * LANES;
  L.A = lds + 3L * m.R * LANES;
  const long t = chem_thread(tiled);
  if (t >= (perm ? (n + GRP - 1) / GRP * GRP : n)) return;   // no block-level synchronisation below
  const long c = bin_cell(perm, t);
  if (c >= n) return;
  const double T = Tf[c], rho_rr = rhof[c];
  double Y0[S], y[S];
#pragma unroll
  for (int i = 0; i < S; ++i) Y0[i] = Yf[(long)i * n + c];
  const double rho = reactor_state<S>(T, pf[c], Y0, m.W, y);
  int steps = 0, rejects = 0;
  double hnext = 0.0;   // the step the integration would take next
  if (T >= Tmin) {
    rate_constants<S>(m, L, T);
    double sc[S];
#pragma unroll
    for (int i = 0; i < S; ++i) sc[i] = rho / m.W[i];   // Y -> C scale for the tolerances
    // first step: the size the previous solve of this cell ended with (OpenFOAM's per-cell deltaTChem)
    const double hp = stats[2 * n + c];
    double t = 0.0, h = hp > 0.0 ? fmin(dt, hp) : dt;
    while (t < dt) {
      if (steps + rejects >= max_steps) { steps = -1; break; }
      if (t + h > dt) h = dt - t;
      double f0[S], r1[S], r2[S], t21[S], t22[S];
      rhs<S>(m, L, T, y, f0);
      bool ok;
      double err = 0.0;
      if (method == 0) {   // ROS3
        ok = ros3<S>(m, L, T, y, f0, h, r2, r1);
        if (ok) {   // weighted RMS error norm (KPP / CVODE)
#pragma unroll
          for (int i = 0; i < S; ++i) {
            const double e = r1[i] / (atol * sc[i] + rtol * fmax(fabs(y[i]), fabs(r2[i])));
            err += e * e;
          }
          err = sqrt(err / S);
          if (!(err == err)) ok = false;
        }
      } else {             // linearly-implicit Euler extrapolation, sequence 1, 2, 3
        ok = lie<S>(m, L, T, y, f0, h, 1, r1);
        ok = ok && lie<S>(m, L, T, y, f0, h, 2, t21);
        if (ok) {
#pragma unroll
          for (int i = 0; i < S; ++i) t22[i] = 2.0 * t21[i] - r1[i];
          ok = lie<S>(m, L, T, y, f0, h, 3, r2);
        }
        if (ok) {
#pragma unroll
          for (int i = 0; i < S; ++i) {
            const double t32 = 3.0 * r2[i] - 2.0 * t21[i];
            const double t33 = t32 + (t32 - t22[i]) * 0.5;
            const double e = fabs(t33 - t32) / (atol * sc[i] + rtol * fabs(t33));
            err = fmax(err, e);
            r2[i] = t33;
          }
          if (!(err == err)) ok = false;   // NaN
        }
      }
      if (ok && err <= 1.0) {
#pragma unroll
        for (int i = 0; i < S; ++i) y[i] = r2[i];
        t += h;
        ++steps;
        const double fac = err > 0.0 ? 0.9 * pow(err, -1.0 / 3.0) : 5.0;
        h = h * fmin(5.0, fmax(0.2, fac));
      } else {
        ++rejects;
        const double fac = ok ? 0.9 * pow(err, -1.0 / 3.0) : 0.25;
        h = h * fmin(0.5, fmax(0.1, fac));
      }
    }
    if (steps >= 0) hnext = h;
  }
  double q = 0.0;   // Qdot = -sum_i hc_i RR_i in species order (dfChemistryModel.C:771)
#pragma unroll
  for (int i = 0; i < S; ++i) {
    const double Yn = y[i] * m.W[i] / rho;
    const double rr = T >= Tmin ? (Yn - Y0[i]) * rho_rr / dt : 0.0;
    RR[(long)i * n + c] = rr;
    q -= hc[i] * rr;
  }
  Qdot[c] = q;
  stats[c] = steps;
  stats[n + c] = rejects;
  if (hnext > 0.0) stats[2 * n + c] = hnext;
  if (steps < 0) atomicAdd(fail, 1);
}

// ---- generated fast path: the mechanism compiled in (dfmi/chem_codegen.py), state in registers
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wunused-variable"
#define DFMI_HD __device__   // the generated kinetics are plain C++; here they run on the device
// between the reactions of the fused rates + Jacobian pass: nothing is scheduled across, so one reaction's
// temporaries die before the next one's loads are issued (the register peak is J plus one reaction)
// (the scheduler left free across reactions measured 13.90 -> 14.11 ms per step, 3 rounds each in one call, round 6)
#define DFMI_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
// 1 / x for the generated kinetics (fall-off factors, LU pivots): the hardware reciprocal estimate refined by two
// Newton steps instead of the ~10-instruction IEEE division sequence (x is a nonzero normal number there)
__device__ __forceinline__ double dfmi_rcp(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  e = fma(-x, r, 1.0);
  return fma(r, e, r);
}
#define DFMI_RCP(x) dfmi_rcp(x)
// products contracted into FMAs inside the generated kinetics (the library builds with -ffp-contract=off for the
// bitwise FV kernels; the chemistry is checked against SciPy BDF to a tolerance, not bitwise)
#define DFMI_CONTRACT() _Pragma("clang fp contract(fast)") do {} while (0)
#include "chem_gen_burke9.inc"
#include "chem_gen_es80.inc"
#pragma clang diagnostic pop

// The integrated state is the mechanism's active species (G::SA; a third-body-only species such as N2 keeps its
// concentration and rides along in y) -- bitwise the full-state integration: the dropped rows and columns
// only ever multiply or add exact zeros (chem_codegen.py).
// Registers: the dense iteration matrix (SA^2 doubles, 128 VGPRs for Burke 9), the state and the stage vectors
// fill the wave's registers, so the NK rate constants -- computed once per cell (T is frozen), read by every
// rate and Jacobian evaluation of the step loop -- live in LDS as [constant][lane] (conflict-free ds_read_b64,
// 24.6 KiB per 64-lane workgroup for Burke 9) instead of 96 more VGPRs that spilled to scratch (round 4:
// 256 VGPR + 256 AGPR + 84 B/lane of scratch at one wave per SIMD).
struct KLds {
  double* base;   // the workgroup's constants, [constant][lane]
  int lane;       // constant i of this lane at base[i * LANES + lane]
  __device__ __forceinline__ double& operator[](int i) const { return base[i * LANES + lane]; }
};

template <class G>
__global__ void __launch_bounds__(LANES, 1) k_chem_gen(long n, const int* __restrict__ perm,
    const double* __restrict__ Tf, const double* __restrict__ pf, const double* __restrict__ rhof,
    const double* __restrict__ Yf, double dt, double rtol, double atol, double Tmin, int max_steps,
    double* __restrict__ RR, double* __restrict__ stats, int* __restrict__ fail, int tiled, const double* __restrict__ hc,
    double* __restrict__ Qdot) {
  constexpr int S = G::S, SA = G::SA;
  constexpr double g = 0.43586652150845899941601945119356;
  constexpr double c21 = -0.10156171083877702091975600115545e1, c31 = 0.40759956452537699824805835358067e1,
                   c32 = 0.92076794298330791242156818474003e1;
  constexpr double m2 = 0.61697947043828245592553615689730e1, m3 = -0.42772256543218573326238373806514;
  constexpr double e1 = 0.5, e2 = -0.29079558716805469821718236208017e1, e3 = 0.22354069897811569627360909276199;
  __shared__ double kl[G::NK * LANES];
  KLds kh{kl, (int)threadIdx.x};
  const long t = chem_thread(tiled);
  if (t >= (perm ? (n + GRP - 1) / GRP * GRP : n)) return;   // no block-level synchronisation below
  const long c = bin_cell(perm, t);
  if (c >= n) return;
  const double T = Tf[c];
  double y[S];
  double rho;
  {
    double Y0[S];
#pragma unroll
    for (int i = 0; i < S; ++i) Y0[i] = Yf[(long)i * n + c];
    rho = reactor_state<S>(T, pf[c], Y0, G::W, y);
  }
  int steps = 0, rejects = 0;
  double hnext = 0.0;   // the step the integration would take next
  if (T >= Tmin) {
    G::consts(T, kh);
    // first step: the size the previous solve of this cell ended with (OpenFOAM's per-cell deltaTChem)
    const double hp = stats[2 * n + c];
    double t = 0.0, h = hp > 0.0 ? fmin(dt, hp) : dt;
    while (t < dt) {
      // the lane offset passes through an empty asm each iteration: the constants' LDS reads cannot be hoisted
      // out of the loop (held in registers across it, which is what this layout exists to avoid)
      asm volatile("" : "+v"(kh.lane));
      double arho = atol * rho;   // tolerance scale atol rho / W_i, formed per use (not 8 values held across the loop)
      asm volatile("" : "+v"(arho));
      if (steps + rejects >= max_steps) { steps = -1; break; }
      if (t + h > dt) h = dt - t;
      const double hg = h * g, rh = dfmi_rcp(h);
      double f0[SA], A[SA * SA];
#pragma unroll
      for (int e = 0; e < SA * SA; ++e) A[e] = 0.0;
      G::wdot_jac(T, kh, y, f0, A);
#pragma unroll
      for (int e = 0; e < SA * SA; ++e) A[e] = (e % (SA + 1) == 0 ? 1.0 : 0.0) - hg * A[e];
      bool ok = G::factor(A);
      double err = 0.0, yn[SA];
      if (ok) {
        double k1[SA], k2[SA], k3[SA], y2[S], f2[SA];
#pragma unroll
        for (int a = 0; a < SA; ++a) k1[a] = hg * f0[a];
        G::solve(A, k1);
#pragma unroll
        for (int i = 0; i < S; ++i) y2[i] = y[i];
#pragma unroll
        for (int a = 0; a < SA; ++a) y2[G::ACT[a]] = y[G::ACT[a]] + k1[a];
        G::wdot(T, kh, y2, f2);
#pragma unroll
        for (int a = 0; a < SA; ++a) k2[a] = hg * (f2[a] + c21 * rh * k1[a]);
        G::solve(A, k2);
#pragma unroll
        for (int a = 0; a < SA; ++a) k3[a] = hg * (f2[a] + rh * (c31 * k1[a] + c32 * k2[a]));
        G::solve(A, k3);
#pragma unroll
        for (int a = 0; a < SA; ++a) {
          const int i = G::ACT[a];
          yn[a] = y[i] + k1[a] + m2 * k2[a] + m3 * k3[a];
          const double e = (e1 * k1[a] + e2 * k2[a] + e3 * k3[a]) * dfmi_rcp(arho * G::RW[i] + rtol * fmax(fabs(y[i]), fabs(yn[a])));
          err += e * e;   // weighted RMS error norm (KPP / CVODE) over all S species (inactive terms are 0)
        }
        err = sqrt(err / S);
        if (!(err == err)) ok = false;
      }
      if (ok && err <= 1.0) {
#pragma unroll
        for (int a = 0; a < SA; ++a) y[G::ACT[a]] = yn[a];
        t += h;
        ++steps;
        const double fac = err > 0.0 ? 0.9 * pow(err, -1.0 / 3.0) : 5.0;
        h = h * fmin(5.0, fmax(0.2, fac));
      } else {
        ++rejects;
        const double fac = ok ? 0.9 * pow(err, -1.0 / 3.0) : 0.25;
        h = h * fmin(0.5, fmax(0.1, fac));
      }
    }
    if (steps >= 0) hnext = h;
  }
  const double rho_rr = rhof[c];   // Y0 and rho_rr re-read here rather than held through the integration
  double q = 0.0;   // Qdot = -sum_i hc_i RR_i in species order (dfChemistryModel.C:771)
#pragma unroll
  for (int i = 0; i < S; ++i) {
    const double Yn = y[i] * G::W[i] / rho;
    const double rr = T >= Tmin ? (Yn - Yf[(long)i * n + c]) * rho_rr / dt : 0.0;
    RR[(long)i * n + c] = rr;
    q -= hc[i] * rr;
  }
  Qdot[c] = q;
  stats[c] = steps;
  stats[n + c] = rejects;
  if (hnext > 0.0) stats[2 * n + c] = hnext;
  if (steps < 0) atomicAdd(fail, 1);
}

// FNV-1a over the packed mechanism, NASA7 rows and molecular weights (dfmi/chem_codegen.py:fingerprint)
unsigned long long fnv(unsigned long long h, const void* p, size_t n) {
  const unsigned char* b = static_cast<const unsigned char*>(p);
  for (size_t i = 0; i < n; ++i) { h ^= b[i]; h *= 0x100000001b3ull; }
  return h;
}

}  // namespace

void chem_upload(Ctx& x, int R, const int* idata, const int* irs, const double* dd) {
  Chem& h = x.chem;
  DFMI_CHECK(x.S > 0 && R > 0 && R <= 256, "chemistry: bad reaction count");
  h.R = R;
  h.ndd = 17 + x.S;
  h.h_idata.assign(idata, idata + (size_t)R * 8);
  h.h_irs.assign(irs, irs + (size_t)R * 6);
  h.h_dd.assign(dd, dd + (size_t)R * (17 + x.S));
  h.idata.upload(idata, (size_t)R * 8, x.stream);
  h.irs.upload(irs, (size_t)R * 6, x.stream);
  h.dd.upload(dd, (size_t)R * h.ndd, x.stream);
  for (int r = 0; r < R; ++r) {
    for (int k = 0; k < 6; ++k) DFMI_CHECK(irs[r * 6 + k] < x.S, "chemistry: species index out of range");
    DFMI_CHECK(idata[r * 8] >= 0 && idata[r * 8] <= 3, "chemistry: unknown reaction type");
  }
  DFMI_HIP(hipStreamSynchronize(x.stream));
  h.ready = true;
}

void chem_solve(Ctx& x, double dt, const char* rho_field) {
  Chem& h = x.chem;
  DFMI_CHECK(h.ready, "chemistry mechanism not set (dfmi_chem_set_mechanism)");
  DFMI_CHECK(x.thermo.S == x.S, "chemistry needs the thermo coefficients (NASA7, W)");
  ChemMech m{h.R, h.ndd, h.idata.p, h.irs.p, h.dd.p, x.thermo.dnasa.p, x.thermo.dW.p};
  const size_t lds = ((size_t)3 * h.R + (size_t)x.S * x.S) * LANES * sizeof(double);
  DFMI_CHECK(lds <= 160 * 1024, "chemistry: mechanism too large for the LDS layout");
  double* stats = x.f("chem_stats");
  const double* rho_rr = x.f(rho_field);
  if (h.fail.n == 0) h.fail.alloc(1);
  if (!h.batch) DFMI_HIP(hipMemsetAsync(h.fail.p, 0, sizeof(int), x.stream));
  h.method = (int)x.opt("chem.method");
  h.bin = (int)x.opt("chem.binning");
  const long ng = (x.C + GRP - 1) / GRP;   // binning groups
  const int tiled = h.bin == 2;
  long nblk = blocks_for(h.bin ? ng * GRP : (long)x.C, LANES);
  if (tiled) nblk = (nblk + 8L * TILE_B - 1) / (8L * TILE_B) * (8L * TILE_B);   // whole groups of 8 tiles
  const dim3 g((unsigned)nblk);
  // compiled-in mechanism? (bitwise the same arrays, NASA7 and weights)
  unsigned long long fp = 0xcbf29ce484222325ull;
  const int S32 = x.S;
  fp = fnv(fp, &S32, 4);
  fp = fnv(fp, h.h_idata.data(), h.h_idata.size() * 4);
  fp = fnv(fp, h.h_irs.data(), h.h_irs.size() * 4);
  fp = fnv(fp, h.h_dd.data(), h.h_dd.size() * 8);
  fp = fnv(fp, x.thermo.nasa.data(), x.thermo.nasa.size() * 8);
  fp = fnv(fp, x.thermo.W.data(), x.thermo.W.size() * 8);
  h.generated = 0;
  if (x.on("chem.generated") && h.method == 0) {
    if (fp == ChemGen_burke9::FINGERPRINT) h.generated = 1;
    else if (fp == ChemGen_es80::FINGERPRINT) h.generated = 2;
  }
  const int* perm = nullptr;
  if (h.bin) {
    KScope _ks(x, "k_bin");
    const int nb = blocks_for(ng, BCELLS);
    if (h.perm.n < (size_t)ng) h.perm.alloc(ng);
    if (h.bcnt.n < (size_t)nb * NBIN) h.bcnt.alloc((size_t)nb * NBIN);
    hipLaunchKernelGGL(k_bin_count, dim3(nb), dim3(BCB), 0, x.stream, (long)x.C, (const double*)stats, nb, h.bcnt.p);
    if (tiled) hipLaunchKernelGGL(k_bin_scan_local, dim3(blocks_for(nb, BCB)), dim3(BCB), 0, x.stream, nb, h.bcnt.p);
    else hipLaunchKernelGGL(k_bin_scan, dim3(1), dim3(1024), 0, x.stream, nb * NBIN, h.bcnt.p);
    hipLaunchKernelGGL(k_bin_scatter, dim3(nb), dim3(BCB), 0, x.stream, (long)x.C, (const double*)stats, nb,
                       (const int*)h.bcnt.p, h.perm.p);
    perm = h.perm.p;
  }
  if (h.generated) {
    KScope _ks(x, "k_chem");
#define GEN(G) hipLaunchKernelGGL((k_chem_gen<G>), g, dim3(LANES), 0, x.stream, (long)x.C, perm, x.f("T"), x.f("p"),  \
                                  rho_rr, x.f("Y"), dt, h.rtol, h.atol, h.Tmin, h.max_steps, x.f("RR"), stats, h.fail.p, tiled,   \
                                  x.thermo.dhc.p, x.f("Qdot"))
    if (h.generated == 1) GEN(ChemGen_burke9); else GEN(ChemGen_es80);
#undef GEN
    DFMI_HIP(hipGetLastError());
    chem_fail_snapshot(x);
    return;
  }
#define CALL(NS)                                                                                                    \
  do {                                                                                                              \
    KScope _ks(x, "k_chem");                                                                                        \
    hipLaunchKernelGGL(k_chem<NS>, g, dim3(LANES), lds, x.stream, (long)x.C, perm, m, x.f("T"), x.f("p"), rho_rr,      \
                       x.f("Y"), dt, h.rtol, h.atol, h.Tmin, h.max_steps, h.method, x.f("RR"), stats, h.fail.p, tiled,   \
                       x.thermo.dhc.p, x.f("Qdot"));                                                          \
  } while (0)
  switch (x.S) {
    case 4: CALL(4); break; case 5: CALL(5); break; case 6: CALL(6); break; case 7: CALL(7); break;
    case 8: CALL(8); break; case 9: CALL(9); break; case 10: CALL(10); break; case 11: CALL(11); break;
    case 12: CALL(12); break;
    default: throw Error("chemistry: species count " + std::to_string(x.S) + " not instantiated (4..12)");
  }
#undef CALL
  DFMI_HIP(hipGetLastError());
  chem_fail_snapshot(x);
}

// The failure count leaves the device behind an event (no stream drain); chem_check reads it at the
// next host synchronisation point the caller already has (end of the time step's solver polls).
void chem_fail_snapshot(Ctx& x) {
  Chem& h = x.chem;
  if (h.batch) return;   // the batch's one snapshot follows its last step
  h.fail_host.ensure(1);
  if (!h.fail_ev) DFMI_HIP(hipEventCreateWithFlags(&h.fail_ev, hipEventDisableTiming));
  DFMI_HIP(hipMemcpyAsync(h.fail_host.p, h.fail.p, sizeof(int), hipMemcpyDeviceToHost, x.stream));
  DFMI_HIP(hipEventRecord(h.fail_ev, x.stream));
  h.fail_pending = true;
}

void chem_check(Ctx& x) {
  Chem& h = x.chem;
  if (!h.fail_pending) return;
  DFMI_HIP(hipEventSynchronize(h.fail_ev));
  h.fail_pending = false;
  const int nf = h.fail_host.p[0];
  DFMI_CHECK(nf == 0, "chemistry: " + std::to_string(nf) + " cell(s)" + (h.batch ? " (summed over the batch's steps)" : "") +
                          " hit the integrator step limit (max_steps = " + std::to_string(h.max_steps) +
                          "); their RR is not a completed integration");
}

}  // namespace dfmi
