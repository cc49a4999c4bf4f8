// thermo.hip -- per-cell thermo/transport update (dfThermo::correctThermo, reference
// src_gpu/dfThermo.cu:54-357, 572-671; CPU semantics dfChemistryModel.C:419-735).
//
// One fused kernel per cell (and one per boundary slot) does what the reference spreads over 8
// launches with intermediate [S][C] arrays: Y->X, mean W, Newton T(h) (atol = rtol = 1e-7, <= 20
// iterations), psi = W/(R T), rho = p psi, Wilke viscosity, mixture conductivity -> alpha = lambda/cp,
// mixture-averaged rhoD_i (Cantera getMixDiffCoeffsMass) and hai_i = h_i(T) (the CPU hai that the
// reference GPU path zeroes, dfYEqn.cu:489-494). The species count is a template parameter so the
// per-cell species arrays stay in VGPRs (runtime-indexed arrays would go to scratch); the coefficient
// tables are wave-uniform reads (scalar cache). HBM traffic per cell: read Y[S], he, p, T;
// write T, he, psi, rho, mu, alpha, rhoD[S], hai[S].
#include "dfmi_ctx.h"
#include <cmath>

namespace dfmi {
namespace {

constexpr double R_GAS = 8314.46261815324;
constexpr double SQRT8 = 2.8284271247461903;

struct TC {   // coefficient table pointers
  const double *W, *nasa, *visc, *cond, *bdiff, *vc1, *vc2;
  int sym;      // bdiff[i][j] == bdiff[j][i] bitwise (binary diffusion fits are symmetric)
};

// NASA7 polynomials of species i at T: cp/R and h/(R T)
__device__ __forceinline__ void nasa_cp_h(const double* a, double T, double& cpR, double& hRT) {
  const int o = (T > a[0]) ? 1 : 8;
  const double T2 = T * T, T3 = T2 * T, T4 = T3 * T;
  cpR = a[o] + a[o + 1] * T + a[o + 2] * T2 + a[o + 3] * T3 + a[o + 4] * T4;
  hRT = a[o] + a[o + 1] * T / 2 + a[o + 2] * T2 / 3 + a[o + 3] * T3 / 4 + a[o + 4] * T4 / 5 + a[o + 5] / T;
}

// mixture h and cp at T, ryw[i] = R Y_i / W_i
template <int S>
__device__ __forceinline__ void hcp_mix(const TC& t, double T, const double* ryw, double& h, double& cp) {
  h = 0.; cp = 0.;
#pragma unroll
  for (int i = 0; i < S; ++i) {
    double c, hh;
    nasa_cp_h(t.nasa + i * 15, T, c, hh);
    h += hh * T * ryw[i];
    cp += c * ryw[i];
  }
}

// state (T or he), p, Y -> T, he, psi, rho, mu, alpha, rhoD[S], hai[S]; mirrors oracle thermo_point
// (same formulas; divisions hoisted out of the O(S^2) loops -- reciprocals of the species
// viscosities, one reciprocal per binary-diffusion pair when the fit table is symmetric -- so the
// result agrees with the sequential evaluation to rounding, not bitwise)
template <int S>
__device__ __forceinline__ void thermo_point(const TC& t, bool fixT, double& T, double& he, double p, const double* y,
                                             double& psi, double& rho, double& mu, double& alpha, double* rhoD,
                                             double* hai) {
  double X[S], rw[S], ryw[S];
  double sum = 0.;
#pragma unroll
  for (int i = 0; i < S; ++i) { rw[i] = R_GAS / t.W[i]; ryw[i] = rw[i] * y[i]; sum += y[i] / t.W[i]; }
  double Wm = 0.;
  const double rsum = 1.0 / sum;
#pragma unroll
  for (int i = 0; i < S; ++i) { X[i] = y[i] / t.W[i] * rsum; Wm += X[i] * t.W[i]; }
  double cpm;
  if (fixT) {
    hcp_mix<S>(t, T, ryw, he, cpm);
  } else {
    double tt = T;
    for (int n = 0; n < 20; ++n) {
      double h, cp;
      hcp_mix<S>(t, tt, ryw, h, cp);
      const double dT = (h - he) / cp;
      tt -= dT;
      if (fabs(h - he) < 1e-7 || fabs(dT / tt) < 1e-7) break;
    }
    T = tt;
    double h_;
    hcp_mix<S>(t, T, ryw, h_, cpm);
  }
  const double lnT = log(T);
  double poly[5];
  poly[0] = 1.0; poly[1] = lnT; poly[2] = poly[1] * poly[1]; poly[3] = poly[1] * poly[2]; poly[4] = poly[2] * poly[2];
  psi = Wm / (R_GAS * T);
  rho = p * psi;
  // Wilke mixture viscosity
  double sv[S], rsv[S], xs[S];
#pragma unroll
  for (int i = 0; i < S; ++i) {
    double dp = 0.;
#pragma unroll
    for (int j = 0; j < 5; ++j) dp += t.visc[i * 5 + j] * poly[j];
    sv[i] = dp;
    rsv[i] = 1.0 / dp;
    xs[i] = X[i] * (1.0 / SQRT8);
  }
  double mumix = 0.;
#pragma unroll
  for (int i = 0; i < S; ++i) {
    double s2 = 0.;
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const double tmp = 1.0 + (sv[i] * rsv[j]) * t.vc2[i * S + j];
      s2 += xs[j] * t.vc1[i * S + j] * (tmp * tmp);
    }
    mumix += X[i] * (sv[i] * sv[i]) / s2;
  }
  const double sT = sqrt(T);
  mu = mumix * sT;
  double sc = 0., sic = 0.;
#pragma unroll
  for (int i = 0; i < S; ++i) {
    double dp = 0.;
#pragma unroll
    for (int j = 0; j < 5; ++j) dp += t.cond[i * 5 + j] * poly[j];
    const double lam = dp * sT;
    sc += X[i] * lam;
    sic += X[i] / lam;
  }
  alpha = 0.5 * (sc + 1.0 / sic) / cpm;
  // mixture-averaged diffusion: s1_i = sum_j X_j / D_ij, s2_i = sum_j X_j W_j / D_ij (j != i, ascending j)
  const double powT = T * sT, rdp = rho / p;
  double s1[S], s2[S];
#pragma unroll
  for (int i = 0; i < S; ++i) { s1[i] = 0.; s2[i] = 0.; }
  if (t.sym) {   // D_ij = D_ji: one fit evaluation and one reciprocal per pair
#pragma unroll
    for (int i = 0; i < S; ++i)
#pragma unroll
      for (int j = i + 1; j < S; ++j) {
        double tmp = 0.;
#pragma unroll
        for (int k = 0; k < 5; ++k) tmp += t.bdiff[(i * S + j) * 5 + k] * poly[k];
        const double inv = 1.0 / (tmp * powT);
        s1[i] += X[j] * inv; s2[i] += X[j] * t.W[j] * inv;
        s1[j] += X[i] * inv; s2[j] += X[i] * t.W[i] * inv;
      }
  } else {
#pragma unroll
    for (int i = 0; i < S; ++i)
#pragma unroll
      for (int j = 0; j < S; ++j) {
        if (i == j) continue;
        double tmp = 0.;
#pragma unroll
        for (int k = 0; k < 5; ++k) tmp += t.bdiff[(i * S + j) * 5 + k] * poly[k];
        const double inv = 1.0 / (tmp * powT);
        s1[i] += X[j] * inv; s2[i] += X[j] * t.W[j] * inv;
      }
  }
#pragma unroll
  for (int i = 0; i < S; ++i) {
    if (X[i] + 1e-10 > 1.) { rhoD[i] = 0.; continue; }
    const double q2 = s2[i] * (X[i] / (Wm - X[i] * t.W[i]));
    rhoD[i] = 1 / (s1[i] + q2) * rdp;
  }
#pragma unroll
  for (int i = 0; i < S; ++i) {
    double c, hh;
    nasa_cp_h(t.nasa + i * 15, T, c, hh);
    hai[i] = hh * T * rw[i];
  }
}

template <int S>
__global__ void __launch_bounds__(256) k_thermo_cells(int n, TC t, int fixT, double* __restrict__ T, double* __restrict__ he,
    const double* __restrict__ p, const double* __restrict__ Y, double* __restrict__ psi, double* __restrict__ rho,
    double* __restrict__ mu, double* __restrict__ alpha, double* __restrict__ rhoD, double* __restrict__ hai) {
  const int c = xcd_block() * blockDim.x + threadIdx.x;
  if (c >= n) return;
  double y[S], rd[S], ha[S];
#pragma unroll
  for (int i = 0; i < S; ++i) y[i] = Y[(long)i * n + c];
  double Tc = T[c], hc = he[c], ps, r, m, a;
  thermo_point<S>(t, fixT != 0, Tc, hc, p[c], y, ps, r, m, a, rd, ha);
  T[c] = Tc; he[c] = hc; psi[c] = ps; rho[c] = r; mu[c] = m; alpha[c] = a;
#pragma unroll
  for (int i = 0; i < S; ++i) { rhoD[(long)i * n + c] = rd[i]; hai[(long)i * n + c] = ha[i]; }
}

// boundary slots: fixedValue T patches evaluate from T (he from T), others from he (CPU
// correctThermo boundary loop, dfChemistryModel.C:560-727); processor [internal n] slots copy cells.
template <int S>
__global__ void __launch_bounds__(256) k_thermo_slots(MeshView m, TC t, const int8_t* __restrict__ tyT, int fromT,
    const double* __restrict__ cT, const double* __restrict__ che, const double* __restrict__ cpsi,
    const double* __restrict__ crho, const double* __restrict__ cmu, const double* __restrict__ calpha,
    const double* __restrict__ crhoD, const double* __restrict__ chai, double* __restrict__ T, double* __restrict__ he,
    const double* __restrict__ p, const double* __restrict__ Y, double* __restrict__ psi, double* __restrict__ rho,
    double* __restrict__ mu, double* __restrict__ alpha, double* __restrict__ rhoD, double* __restrict__ hai) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  const int B = m.B;
  if (b >= B) return;
  const int ty = tyT[b];
  if (ty == EMPTY) return;
  if (bc_proc(ty) && !m.sprim[b]) {
    const int c = m.bfc[b];
    const long C = m.C;
    T[b] = cT[c]; he[b] = che[c]; psi[b] = cpsi[c]; rho[b] = crho[c]; mu[b] = cmu[c]; alpha[b] = calpha[c];
#pragma unroll
    for (int i = 0; i < S; ++i) { rhoD[(long)i * B + b] = crhoD[i * C + c]; hai[(long)i * B + b] = chai[i * C + c]; }
    return;
  }
  double y[S], rd[S], ha[S];
#pragma unroll
  for (int i = 0; i < S; ++i) y[i] = Y[(long)i * B + b];
  double Tb = T[b], hb = he[b], ps, r, mm, a;
  thermo_point<S>(t, fromT != 0 || bc_fixes_value(ty), Tb, hb, p[b], y, ps, r, mm, a, rd, ha);
  T[b] = Tb; he[b] = hb; psi[b] = ps; rho[b] = r; mu[b] = mm; alpha[b] = a;
#pragma unroll
  for (int i = 0; i < S; ++i) { rhoD[(long)i * B + b] = rd[i]; hai[(long)i * B + b] = ha[i]; }
}

// mixture enthalpy summed exactly as calculate_enthalpy_device_kernel (dfThermo.cu:257-274) and the
// oracle's h_mix do it (same operation order: the energy gradient is compared bitwise)
template <int S>
__device__ __forceinline__ double h_ref(const TC& t, double T, const double* y, long ys) {
  double h = 0.;
#pragma unroll
  for (int i = 0; i < S; ++i) {
    const double* a = t.nasa + i * 15;
    const int o = (T > a[0]) ? 1 : 8;
    h += (a[o] + a[o + 1] * T / 2 + a[o + 2] * T * T / 3 + a[o + 3] * T * T * T / 4 + a[o + 4] * T * T * T * T / 5 +
          a[o + 5] / T) * R_GAS * T / t.W[i] * y[i * ys];
  }
  return h;
}

// calculate_energy_gradient_kernel (dfThermo.cu:276-294): on gradientEnergy slots of he,
// (h(T_c, Y_b) - h(T_c, Y_c)) * deltaCoeffs; 0 on every other slot
template <int S>
__global__ void k_energy_gradient(MeshView m, TC t, const int8_t* __restrict__ tyH, const double* __restrict__ T,
                                  const double* __restrict__ Y, const double* __restrict__ bY, double* __restrict__ eg) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= m.B) return;
  if (tyH[b] != GRADIENT_ENERGY) { eg[b] = 0.0; return; }
  const int c = m.bfc[b];
  const double Tc = T[c];
  const double hb = h_ref<S>(t, Tc, bY + b, m.B), hc = h_ref<S>(t, Tc, Y + c, m.C);
  eg[b] = (hb - hc) * m.bdc[b];
}


// ---------------------------------------------------------------- large mechanisms (S > 16)
// One cell per group of TG = 16 lanes (4 cells per wave, 16 per workgroup): lane l owns species
// l, l + 16, l + 32, l + 48 in registers; the O(S^2) Wilke and mixture-averaged-diffusion rows are
// split over the lanes, reading the cell's mole fractions and species viscosities from LDS; mixture
// sums are butterfly reductions inside the group (every lane ends with the identical value, so the
// Newton iteration and the group's control flow stay uniform). Same formulas as thermo_point; only
// the summation order of the mixture sums differs (agrees with the sequential oracle to rounding).
constexpr int TG = 16, TCB = 256, TCELLS = TCB / TG, SMAX = 64, SPL = SMAX / TG;

__device__ __forceinline__ double gsum(double v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  v += __shfl_xor(v, 8, 64);
  return v;
}

// slots == nullptr: cells (index = cell, stride n); otherwise boundary slots with per-slot types
__global__ void __launch_bounds__(TCB) k_thermo_coop(int n, int S, TC t, int fixT_all, const int8_t* __restrict__ ty,
    const int8_t* __restrict__ sprim, const int* __restrict__ bfc, long Cc, const double* __restrict__ cT,
    const double* __restrict__ che, const double* __restrict__ cpsi, const double* __restrict__ crho,
    const double* __restrict__ cmu, const double* __restrict__ calpha, const double* __restrict__ crhoD,
    const double* __restrict__ chai, double* __restrict__ T, double* __restrict__ he, const double* __restrict__ p,
    const double* __restrict__ Y, double* __restrict__ psi, double* __restrict__ rho, double* __restrict__ mu,
    double* __restrict__ alpha, double* __restrict__ rhoD, double* __restrict__ hai) {
  __shared__ double sX[TCELLS][SMAX], sS[TCELLS][SMAX], sR[TCELLS][SMAX];
  const int grp = threadIdx.x / TG, l = threadIdx.x % TG;
  const int blk = ty ? (int)blockIdx.x : xcd_block();
  const int idx = blk * TCELLS + grp;
  bool live = idx < n;
  bool fixT = fixT_all != 0;
  if (live && ty) {
    const int tt = ty[idx];
    if (tt == EMPTY) live = false;
    else if (bc_proc(tt) && !sprim[idx]) {   // processor [internal n] slot: copy the cell's values
      const int c = bfc[idx];
      if (l == 0) { T[idx] = cT[c]; he[idx] = che[c]; psi[idx] = cpsi[c]; rho[idx] = crho[c]; mu[idx] = cmu[c]; alpha[idx] = calpha[c]; }
      for (int i = l; i < S; i += TG) { rhoD[(long)i * n + idx] = crhoD[i * Cc + c]; hai[(long)i * n + idx] = chai[i * Cc + c]; }
      live = false;
    } else if (bc_fixes_value(tt)) fixT = true;
  }
  // species owned by this lane; groups without work evaluate a dummy state (uniform barriers below)
  double y[SPL], X[SPL], ryw[SPL];
  double sum = 0.0;
#pragma unroll
  for (int q = 0; q < SPL; ++q) {
    const int i = q * TG + l;
    y[q] = (i < S) ? (live ? Y[(long)i * n + idx] : (i == 0 ? 1.0 : 0.0)) : 0.0;
    if (i < S) sum += y[q] / t.W[i];
  }
  sum = gsum(sum);
  const double rsum = 1.0 / sum;
  double wm = 0.0;
#pragma unroll
  for (int q = 0; q < SPL; ++q) {
    const int i = q * TG + l;
    X[q] = i < S ? y[q] / t.W[i] * rsum : 0.0;
    ryw[q] = i < S ? R_GAS / t.W[i] * y[q] : 0.0;
    if (i < S) wm += X[q] * t.W[i];
  }
  const double Wm = gsum(wm);
  double Tc = live ? T[idx] : 300.0, hc = live ? he[idx] : 0.0;
  const double pc = live ? p[idx] : 101325.0;
  if (!live) fixT = true;
  auto hcp = [&](double TT, double& h, double& cp) {
    double hh = 0.0, cc = 0.0;
#pragma unroll
    for (int q = 0; q < SPL; ++q) {
      const int i = q * TG + l;
      if (i < S) {
        double c1, h1;
        nasa_cp_h(t.nasa + i * 15, TT, c1, h1);
        hh += h1 * TT * ryw[q];
        cc += c1 * ryw[q];
      }
    }
    h = gsum(hh);
    cp = gsum(cc);
  };
  double cpm;
  if (fixT) {
    hcp(Tc, hc, cpm);
  } else {
    double tt = Tc;
    for (int it = 0; it < 20; ++it) {
      double h, cp;
      hcp(tt, h, cp);
      const double dT = (h - hc) / cp;
      tt -= dT;
      if (fabs(h - hc) < 1e-7 || fabs(dT / tt) < 1e-7) break;
    }
    Tc = tt;
    double h_;
    hcp(Tc, h_, cpm);
  }
  const double lnT = log(Tc);
  double poly[5];
  poly[0] = 1.0; poly[1] = lnT; poly[2] = poly[1] * poly[1]; poly[3] = poly[1] * poly[2]; poly[4] = poly[2] * poly[2];
  const double ps = Wm / (R_GAS * Tc);
  const double rh = pc * ps;
  double sv[SPL];
#pragma unroll
  for (int q = 0; q < SPL; ++q) {
    const int i = q * TG + l;
    double dp = 0.0;
    if (i < S)
#pragma unroll
      for (int j = 0; j < 5; ++j) dp += t.visc[i * 5 + j] * poly[j];
    sv[q] = dp;
    if (i < S) { sX[grp][i] = X[q] * (1.0 / SQRT8); sS[grp][i] = dp; sR[grp][i] = 1.0 / dp; }
  }
  __syncthreads();
  // Wilke rows
  double mpart = 0.0;
#pragma unroll
  for (int q = 0; q < SPL; ++q) {
    const int i = q * TG + l;
    if (i >= S) break;
    double s2 = 0.0;
    for (int j = 0; j < S; ++j) {
      const double tmp = 1.0 + (sv[q] * sR[grp][j]) * t.vc2[i * S + j];
      s2 += sX[grp][j] * t.vc1[i * S + j] * (tmp * tmp);
    }
    mpart += X[q] * (sv[q] * sv[q]) / s2;
  }
  const double sT = sqrt(Tc);
  const double mum = gsum(mpart) * sT;
  double sc = 0.0, sic = 0.0;
#pragma unroll
  for (int q = 0; q < SPL; ++q) {
    const int i = q * TG + l;
    if (i >= S) break;
    double dp = 0.0;
#pragma unroll
    for (int j = 0; j < 5; ++j) dp += t.cond[i * 5 + j] * poly[j];
    const double lam = dp * sT;
    sc += X[q] * lam;
    sic += X[q] / lam;
  }
  sc = gsum(sc);
  sic = gsum(sic);
  const double al = 0.5 * (sc + 1.0 / sic) / cpm;
  __syncthreads();   // mole fractions (unscaled) for the diffusion rows
#pragma unroll
  for (int q = 0; q < SPL; ++q) {
    const int i = q * TG + l;
    if (i < S) sX[grp][i] = X[q];
  }
  __syncthreads();
  const double powT = Tc * sT, rdp = rh / pc;
  double rd[SPL], ha[SPL];
#pragma unroll
  for (int q = 0; q < SPL; ++q) {
    const int i = q * TG + l;
    rd[q] = 0.0; ha[q] = 0.0;
    if (i >= S) continue;
    if (!(X[q] + 1e-10 > 1.)) {
      double s1 = 0.0, s2 = 0.0;
      for (int j = 0; j < S; ++j) {
        if (j == i) continue;
        const double* bd = t.bdiff + (i * S + j) * 5;
        const double tmp = bd[0] * poly[0] + bd[1] * poly[1] + bd[2] * poly[2] + bd[3] * poly[3] + bd[4] * poly[4];
        const double inv = 1.0 / (tmp * powT);
        const double xj = sX[grp][j];
        s1 += xj * inv;
        s2 += xj * t.W[j] * inv;
      }
      const double q2 = s2 * (X[q] / (Wm - X[q] * t.W[i]));
      rd[q] = 1 / (s1 + q2) * rdp;
    }
    double c1, h1;
    nasa_cp_h(t.nasa + i * 15, Tc, c1, h1);
    ha[q] = h1 * Tc * (R_GAS / t.W[i]);
  }
  if (!live) return;
  if (l == 0) { T[idx] = Tc; he[idx] = hc; psi[idx] = ps; rho[idx] = rh; mu[idx] = mum; alpha[idx] = al; }
#pragma unroll
  for (int q = 0; q < SPL; ++q) {
    const int i = q * TG + l;
    if (i < S) { rhoD[(long)i * n + idx] = rd[q]; hai[(long)i * n + idx] = ha[q]; }
  }
}

// runtime-S energy gradient (same summation as h_ref: bitwise the template's)
__device__ __forceinline__ double h_ref_rt(const TC& t, int S, double T, const double* y, long ys) {
  double h = 0.;
  for (int i = 0; i < S; ++i) {
    const double* a = t.nasa + i * 15;
    const int o = (T > a[0]) ? 1 : 8;
    h += (a[o] + a[o + 1] * T / 2 + a[o + 2] * T * T / 3 + a[o + 3] * T * T * T / 4 + a[o + 4] * T * T * T * T / 5 +
          a[o + 5] / T) * R_GAS * T / t.W[i] * y[i * ys];
  }
  return h;
}
__global__ void k_energy_gradient_rt(MeshView m, int S, TC t, const int8_t* __restrict__ tyH, const double* __restrict__ T,
                                     const double* __restrict__ Y, const double* __restrict__ bY, double* __restrict__ eg) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= m.B) return;
  if (tyH[b] != GRADIENT_ENERGY) { eg[b] = 0.0; return; }
  const int c = m.bfc[b];
  const double Tc = T[c];
  const double hb = h_ref_rt(t, S, Tc, bY + b, m.B), hc = h_ref_rt(t, S, Tc, Y + c, m.C);
  eg[b] = (hb - hc) * m.bdc[b];
}

}  // namespace

void thermo_upload(Ctx& x) {
  Thermo& t = x.thermo;
  t.dW.upload(t.W, x.stream);
  t.dnasa.upload(t.nasa, x.stream);
  t.dvisc.upload(t.visc, x.stream);
  t.dcond.upload(t.cond, x.stream);
  t.dbdiff.upload(t.bdiff, x.stream);
  t.dvc1.upload(t.vc1, x.stream);
  t.dvc2.upload(t.vc2, x.stream);
}

void thermo_energy_gradient(Ctx& x) {
  Thermo& th = x.thermo;
  DFMI_CHECK(th.S == x.S, "thermo coefficients not set or species count mismatch");
  if (x.B == 0) return;
  const auto& pt = x.pt("he");
  bool any = false;
  for (int p = 0; p < x.P; ++p) any = any || pt[p] == GRADIENT_ENERGY;
  if (!any) return;   // the field stays zero
  TC t{th.dW, th.dnasa, th.dvisc, th.dcond, th.dbdiff, th.dvc1, th.dvc2, 0};
  MeshView m = x.view();
#define CALL(NS)                                                                                                  \
  hipLaunchKernelGGL(k_energy_gradient<NS>, dim3(blocks_for(x.B, 256)), dim3(256), 0, x.stream, m, t, x.st("he"), \
                     x.f("T"), x.f("Y"), x.f("boundary_Y"), x.f("boundary_heGradient"))
  if (species_generic(x.S))
    hipLaunchKernelGGL(k_energy_gradient_rt, dim3(blocks_for(x.B, 256)), dim3(256), 0, x.stream, m, x.S, t, x.st("he"),
                       x.f("T"), x.f("Y"), x.f("boundary_Y"), x.f("boundary_heGradient"));
  else switch (x.S) {
    case 2: CALL(2); break; case 3: CALL(3); break; case 4: CALL(4); break; case 5: CALL(5); break;
    case 6: CALL(6); break; case 7: CALL(7); break; case 8: CALL(8); break; case 9: CALL(9); break;
    case 10: CALL(10); break; case 11: CALL(11); break; case 12: CALL(12); break; case 13: CALL(13); break;
    case 14: CALL(14); break; case 15: CALL(15); break; case 16: CALL(16); break;
    default: throw Error("dfmi: thermo species count " + std::to_string(x.S) + " not supported");
  }
#undef CALL
  DFMI_HIP(hipGetLastError());
}

void thermo_correct(Ctx& x, bool from_T) {
  Thermo& th = x.thermo;
  DFMI_CHECK(th.S == x.S, "thermo coefficients not set or species count mismatch");
  int sym = 1;
  for (int i = 0; i < th.S && sym; ++i)
    for (int j = 0; j < th.S && sym; ++j)
      for (int k = 0; k < 5; ++k)
        if (th.bdiff[(i * th.S + j) * 5 + k] != th.bdiff[(j * th.S + i) * 5 + k]) { sym = 0; break; }
  TC t{th.dW, th.dnasa, th.dvisc, th.dcond, th.dbdiff, th.dvc1, th.dvc2, sym};
  MeshView m = x.view();
#define CALL(NS)                                                                                                   \
  do {                                                                                                            \
    if (x.C > 0) { KScope _ks(x, "k_thermo_cells"); hipLaunchKernelGGL(k_thermo_cells<NS>, dim3(blocks_for(x.C, 256)), dim3(256), 0, x.stream, x.C, t, \
                       (int)from_T, x.f("T"), x.f("he"), x.f("p"), x.f("Y"), x.f("psi"), x.f("rho"), x.f("mu"),    \
                       x.f("alpha"), x.f("rhoD"), x.f("hai")); }                                                  \
    DFMI_HIP(hipGetLastError());                                                                                  \
    if (x.B > 0) hipLaunchKernelGGL(k_thermo_slots<NS>, dim3(blocks_for(x.B, 256)), dim3(256), 0, x.stream, m, t,  \
                       x.st("T"), (int)from_T, x.f("T"), x.f("he"), x.f("psi"), x.f("rho"), x.f("mu"), x.f("alpha"), \
                       x.f("rhoD"), x.f("hai"), x.f("boundary_T"), x.f("boundary_he"), x.f("boundary_p"),          \
                       x.f("boundary_Y"), x.f("boundary_psi"), x.f("boundary_rho"), x.f("boundary_mu"),            \
                       x.f("boundary_alpha"), x.f("boundary_rhoD"), x.f("boundary_hai"));                         \
    DFMI_HIP(hipGetLastError());                                                                                  \
  } while (0)
  if (species_generic(x.S)) {
    DFMI_CHECK(x.S <= SMAX, "thermo: at most 64 species");
    if (x.C > 0) {
      KScope _ks(x, "k_thermo_cells");
      hipLaunchKernelGGL(k_thermo_coop, dim3(blocks_for(x.C, TCELLS)), dim3(TCB), 0, x.stream, x.C, x.S, t, (int)from_T,
                         (const int8_t*)nullptr, (const int8_t*)nullptr, (const int*)nullptr, 0L, (const double*)nullptr,
                         (const double*)nullptr, (const double*)nullptr, (const double*)nullptr, (const double*)nullptr,
                         (const double*)nullptr, (const double*)nullptr, (const double*)nullptr, x.f("T"), x.f("he"),
                         x.f("p"), x.f("Y"), x.f("psi"), x.f("rho"), x.f("mu"), x.f("alpha"), x.f("rhoD"), x.f("hai"));
    }
    DFMI_HIP(hipGetLastError());
    if (x.B > 0)
      hipLaunchKernelGGL(k_thermo_coop, dim3(blocks_for(x.B, TCELLS)), dim3(TCB), 0, x.stream, x.B, x.S, t, (int)from_T,
                         x.st("T"), m.sprim, m.bfc, (long)x.C, x.f("T"), x.f("he"), x.f("psi"), x.f("rho"), x.f("mu"),
                         x.f("alpha"), x.f("rhoD"), x.f("hai"), x.f("boundary_T"), x.f("boundary_he"),
                         x.f("boundary_p"), x.f("boundary_Y"), x.f("boundary_psi"), x.f("boundary_rho"),
                         x.f("boundary_mu"), x.f("boundary_alpha"), x.f("boundary_rhoD"), x.f("boundary_hai"));
    DFMI_HIP(hipGetLastError());
  } else switch (x.S) {
    case 2: CALL(2); break; case 3: CALL(3); break; case 4: CALL(4); break; case 5: CALL(5); break;
    case 6: CALL(6); break; case 7: CALL(7); break; case 8: CALL(8); break; case 9: CALL(9); break;
    case 10: CALL(10); break; case 11: CALL(11); break; case 12: CALL(12); break; case 13: CALL(13); break;
    case 14: CALL(14); break; case 15: CALL(15); break; case 16: CALL(16); break;
    default: throw Error("dfmi: thermo species count " + std::to_string(x.S) + " not supported");
  }
#undef CALL
  // neighbour halves of the processor slots carry the neighbour rank's cell values
  if (from_T) halo_fields(x, {"he", "T", "psi", "rho", "mu", "alpha", "rhoD", "hai"});
  else halo_fields(x, {"T", "psi", "rho", "mu", "alpha", "rhoD", "hai"});
}

}  // namespace dfmi
