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
#include <cstdlib>
#include <cmath>

namespace dfmi {
namespace {

constexpr double R_GAS = 8314.46261815324;
constexpr double SQRT8 = 2.8284271247461903;

struct TC {   // coefficient table pointers
  const double *W, *rW, *nasa, *visc, *cond, *bdiff, *vc1, *vc2;   // rW = 1 / W
  int sym;      // bdiff[i][j] == bdiff[j][i] bitwise (binary diffusion fits are symmetric)
  const double *nasaT, *bdiffT, *vc1T, *vc2T;   // species-minor copies (Thermo::dnasaT ...), coop kernel
  const double *vcP, *bdR;                      // packed copies (Thermo::dvcP, dbdR; bdR only when sym)
};

// 1/x from the hardware reciprocal estimate refined by two Newton steps (correctly rounded in all but rare
// last-bit cases; x is a positive normal number here): a short dependency chain in place of the IEEE division
// sequence (~10 instructions)
__device__ __forceinline__ double rcp_nr(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  e = fma(-x, r, 1.0);
  return fma(r, e, r);
}

// powers of T shared by the S species' NASA7 evaluations at one temperature: the divisions by 3, 5 and T once
// per temperature instead of once per species (the result agrees with the per-species divisions to rounding)
struct TPow { double T, T2, T3, T4, H1, H2, H3, H4, RT; };
__device__ __forceinline__ TPow tpow(double T) {
  const double T2 = T * T, T3 = T2 * T, T4 = T3 * T;
  return TPow{T, T2, T3, T4, T * 0.5, T2 * (1.0 / 3.0), T3 * 0.25, T4 * (1.0 / 5.0), rcp_nr(T)};
}
// NASA7 polynomials of species i at T: cp/R and h/(R T)
__device__ __forceinline__ void nasa_cp_h(const double* a, const TPow& q, double& cpR, double& hRT) {
  const int o = (q.T > a[0]) ? 1 : 8;
  const double a0 = a[o], a1 = a[o + 1], a2 = a[o + 2], a3 = a[o + 3], a4 = a[o + 4], a5 = a[o + 5];
  cpR = a0 + a1 * q.T + a2 * q.T2 + a3 * q.T3 + a4 * q.T4;
  hRT = a0 + a1 * q.H1 + a2 * q.H2 + a3 * q.H3 + a4 * q.H4 + a5 * q.RT;
}

// mixture h and cp at T, ryw[i] = R Y_i / W_i
template <int S>
__device__ __forceinline__ void hcp_mix(const TC& t, double T, const double* ryw, double& h, double& cp) {
  const TPow q = tpow(T);
  h = 0.; cp = 0.;
#pragma unroll
  for (int i = 0; i < S; ++i) {
    double c, hh;
    nasa_cp_h(t.nasa + i * 15, q, c, hh);
    h += hh * T * ryw[i];
    cp += c * ryw[i];
  }
}

// Which outputs one evaluation produces: the whole update (TH_ALL), the state the pressure equation needs
// (TH_STATE: T, he, psi, rho) or the transport the next time step's equations need (TH_TRANSPORT: mu, alpha,
// rhoD, hai at the given T; rhoD's rho / p is psi there, equal to rounding -- p and rho are the pressure
// corrector's while the transport runs beside it)
enum { TH_ALL = 0, TH_STATE = 1, TH_TRANSPORT = 2 };

// state (T or he), p, Y -> T, he, psi, rho, mu, alpha, rhoD[S], hai[S]; mirrors oracle thermo_point
// (same formulas; divisions hoisted out of the O(S^2) loops -- reciprocals of the species
// viscosities, one reciprocal per binary-diffusion pair when the fit table is symmetric -- and the
// per-species divisions as products with 1/W, T powers shared per temperature (tpow) and Newton-refined
// reciprocals (rcp_nr), so the result agrees with the sequential evaluation to rounding, not bitwise;
// the Newton step and its stopping test keep their divisions, so the iteration count is the oracle's)
template <int S, int PART = TH_ALL>
__device__ __forceinline__ void thermo_point(const TC& t, bool fixT, double& T, double& he, double p, const double* y,
                                             double& psi, double& rho, double& mu, double& alpha, double* rhoD,
                                             double* hai) {
  // products contracted into FMAs (the result agrees with the oracle to rounding either way): ~30 % fewer
  // VALU instructions in the O(S^2) rows of this FP64-issue-bound kernel
#pragma clang fp contract(fast)
  double X[S], rw[S], ryw[S];
  double sum = 0.;
#pragma unroll
  for (int i = 0; i < S; ++i) { rw[i] = R_GAS * t.rW[i]; ryw[i] = rw[i] * y[i]; sum += y[i] * t.rW[i]; }
  double Wm = 0.;
  const double rsum = 1.0 / sum;
#pragma unroll
  for (int i = 0; i < S; ++i) { X[i] = y[i] * t.rW[i] * rsum; Wm += X[i] * t.W[i]; }
  double cpm = 0.;
  if (PART == TH_TRANSPORT) {   // T given: only the mixture cp (alpha's), as the fixT branch computes it
    double h_;
    hcp_mix<S>(t, T, ryw, h_, cpm);
  } else if (fixT) {
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
  if (PART == TH_STATE) { rho = p * psi; return; }
  if (PART == TH_ALL) rho = p * psi;
  // Wilke mixture viscosity
  double sv[S], rsv[S], xs[S];
#pragma unroll
  for (int i = 0; i < S; ++i) {
    double dp = 0.;
#pragma unroll
    for (int j = 0; j < 5; ++j) dp += t.visc[i * 5 + j] * poly[j];
    sv[i] = dp;
    rsv[i] = rcp_nr(dp);
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
    mumix += X[i] * (sv[i] * sv[i]) * rcp_nr(s2);
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
    sic += X[i] * rcp_nr(lam);
  }
  alpha = 0.5 * (sc + 1.0 / sic) / cpm;
  // mixture-averaged diffusion: s1_i = sum_j X_j / D_ij, s2_i = sum_j X_j W_j / D_ij (j != i, ascending j)
  const double powT = T * sT, rdp = PART == TH_TRANSPORT ? psi : rho / p;
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
        const double inv = rcp_nr(tmp * powT);
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
    const double q2 = s2[i] * (X[i] * rcp_nr(Wm - X[i] * t.W[i]));
    rhoD[i] = rcp_nr(s1[i] + q2) * rdp;
  }
  const TPow qT = tpow(T);
#pragma unroll
  for (int i = 0; i < S; ++i) {
    double c, hh;
    nasa_cp_h(t.nasa + i * 15, qT, c, hh);
    hai[i] = hh * T * rw[i];
  }
}

// Register budget: S <= 9 is compiled for 3 waves per SIMD (S = 9: 167 VGPRs with 20 B/lane of spill when this was
// set, 162 and none on the round-6 tree, against the compiler's own 172 VGPRs / 2 waves): k_thermo_cells<9>
// 506-508 -> 460-462 us on the 2M headline
// (profiles/r04_thermo_waves_ab.json, two runs each). Larger register-resident mechanisms keep the compiler's choice.
// The transport half alone (TH_TRANSPORT) spills ~380 B/lane at that cap (its Wilke and diffusion rows keep the
// whole X / sv / s1 / s2 set live with nothing to retire early), so it is compiled for 2 waves: it runs beside
// the p solve, where occupancy is not what bounds it (256 VGPRs, no scratch).
template <int S, int PART = 0> constexpr int thermo_wv() { return S <= 9 ? (PART == 2 ? 2 : 3) : 1; }

// T/he/psi/rho written unless PART is TH_TRANSPORT, mu/alpha/rhoD/hai unless it is TH_STATE
template <int S, int PART>
__device__ __forceinline__ void thermo_store(long i0, long n, double* T, double* he, double* psi, double* rho, double* mu,
    double* alpha, double* rhoD, double* hai, double Tv, double hv, double ps, double r, double m, double a,
    const double* rd, const double* ha) {
  if (PART != TH_TRANSPORT) { T[i0] = Tv; he[i0] = hv; psi[i0] = ps; rho[i0] = r; }
  if (PART != TH_STATE) {
    mu[i0] = m; alpha[i0] = a;
#pragma unroll
    for (int i = 0; i < S; ++i) { rhoD[(long)i * n + i0] = rd[i]; hai[(long)i * n + i0] = ha[i]; }
  }
}

template <int S, int PART>
__global__ void __launch_bounds__(256, (thermo_wv<S, PART>())) k_thermo_cells(int n, TC t, int fixT, double* __restrict__ T, double* __restrict__ he,
    const double* __restrict__ p, const double* __restrict__ Y, double* __restrict__ psi, double* __restrict__ rho,
    double* __restrict__ mu, double* __restrict__ alpha, double* __restrict__ rhoD, double* __restrict__ hai) {
  const int c = xcd_block() * blockDim.x + threadIdx.x;
  if (c >= n) return;
  double y[S], rd[S], ha[S];
#pragma unroll
  for (int i = 0; i < S; ++i) y[i] = Y[(long)i * n + c];
  double Tc = T[c], hc = PART == TH_TRANSPORT ? 0. : he[c], ps, r, m, a;
  thermo_point<S, PART>(t, PART == TH_TRANSPORT || fixT != 0, Tc, hc, PART == TH_TRANSPORT ? 0. : p[c], y, ps, r, m, a,
                        rd, ha);
  thermo_store<S, PART>(c, n, T, he, psi, rho, mu, alpha, rhoD, hai, Tc, hc, ps, r, m, a, rd, ha);
}

// boundary slots: fixedValue T patches evaluate from T (he from T), others from he (CPU
// correctThermo boundary loop, dfChemistryModel.C:560-727); processor [internal n] slots copy cells.
template <int S, int PART>
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
    if (PART != TH_TRANSPORT) { T[b] = cT[c]; he[b] = che[c]; psi[b] = cpsi[c]; rho[b] = crho[c]; }
    if (PART != TH_STATE) {
      mu[b] = cmu[c]; alpha[b] = calpha[c];
#pragma unroll
      for (int i = 0; i < S; ++i) { rhoD[(long)i * B + b] = crhoD[i * C + c]; hai[(long)i * B + b] = chai[i * C + c]; }
    }
    return;
  }
  double y[S], rd[S], ha[S];
#pragma unroll
  for (int i = 0; i < S; ++i) y[i] = Y[(long)i * B + b];
  double Tb = T[b], hb = PART == TH_TRANSPORT ? 0. : he[b], ps, r, mm, a;
  thermo_point<S, PART>(t, PART == TH_TRANSPORT || fromT != 0 || bc_fixes_value(ty), Tb, hb,
                        PART == TH_TRANSPORT ? 0. : p[b], y, ps, r, mm, a, rd, ha);
  thermo_store<S, PART>(b, B, T, he, psi, rho, mu, alpha, rhoD, hai, Tb, hb, ps, r, mm, a, rd, ha);
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
// A group of TG = 16 lanes evaluates NCB cells together: lane l owns species l, l + 16, l + 32,
// l + 48 of all NCB cells in registers. The O(S^2) Wilke and mixture-averaged-diffusion rows are
// split over the lanes; every pair-coefficient load (vc1, vc2, the 5 binary-diffusion fit
// coefficients, from the species-minor tables so a group's load is one contiguous run) is used by
// the NCB cells at once -- with one cell per group the kernel was bound by those loads through the
// vector L1 (measured 13 ms per 2M cells x 53 species). The cells' mole fractions and species
// viscosities sit in LDS; mixture sums are butterfly reductions inside the group (every lane ends
// with the identical value, so each cell's Newton iteration and control flow stay uniform over its
// group). Same formulas as thermo_point; the summation order of the mixture sums and the
// contraction of the polynomial products into FMAs differ (agrees with the sequential oracle to
// rounding: the tests hold it to 1e-12).
constexpr int TCB = 256, SMAX = 64;

// Sum over the group, every lane ending with the same bits (one wave: wave_sum, dfmi_common.h)
template <int TG>
__device__ __forceinline__ double gsum(double v) {
  if constexpr (TG == 64) {
    v = wave_sum(v);
    return v;
  } else {
#pragma unroll
    for (int o = 1; o < TG; o <<= 1) v += __shfl_xor(v, o, 64);
    return v;
  }
}


// a group's own LDS rows written and read back by its own lanes: a wave-level ordering when the group is one wave
template <int TG>
__device__ __forceinline__ void group_sync() {
  if constexpr (TG == 64) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else {
    __syncthreads();
  }
}

// slots == nullptr: cells (index = cell, stride n); otherwise boundary slots with per-slot types
template <int TG, int NCB>
__global__ void __launch_bounds__(TCB) k_thermo_coop(int n, int S, TC t, int fixT_all, const int8_t* __restrict__ ty,
    const int8_t* __restrict__ sprim, const int* __restrict__ bfc, long Cc, const double* __restrict__ cT,
    const double* __restrict__ che, const double* __restrict__ cpsi, const double* __restrict__ crho,
    const double* __restrict__ cmu, const double* __restrict__ calpha, const double* __restrict__ crhoD,
    const double* __restrict__ chai, double* __restrict__ T, double* __restrict__ he, const double* __restrict__ p,
    const double* __restrict__ Y, double* __restrict__ psi, double* __restrict__ rho, double* __restrict__ mu,
    double* __restrict__ alpha, double* __restrict__ rhoD, double* __restrict__ hai) {
#pragma clang fp contract(fast)
  constexpr int GPB = TCB / TG, SPL = SMAX / TG;      // groups per block, species per lane
  constexpr int CPB = GPB * NCB;                      // cells per block
  // per-cell rows (+1: groups on distinct banks); a group only touches its own NCB rows except in the
  // block-wide transposes that load Y and store rhoD/hai with cell-contiguous (coalesced) accesses
  __shared__ double sX[CPB][SMAX + 1], sR[CPB][SMAX + 1];
  __shared__ double2 sP[CPB][SMAX];   // Wilke rows: {x_j / sqrt 8, 1 / sv_j}, one 16-B broadcast read per pair
  __shared__ int sLive[CPB];
  const int grp = threadIdx.x / TG, l = threadIdx.x % TG;
  const int DS = (S / 2) * S;
  const double2* vcP = reinterpret_cast<const double2*>(t.vcP);
  const double2* bdp = reinterpret_cast<const double2*>(t.bdR);
  const int blk = ty ? (int)blockIdx.x : xcd_block();
  const long base = (long)blk * CPB;
  for (int e = threadIdx.x; e < CPB * S; e += TCB) {
    const int sp = e / CPB, cl = e % CPB;
    sX[cl][sp] = base + cl < n ? Y[(long)sp * n + base + cl] : 0.0;
  }
  __syncthreads();
  int idx[NCB];
  bool live[NCB], fixT[NCB];
#pragma unroll
  for (int c = 0; c < NCB; ++c) {
    idx[c] = (blk * GPB + grp) * NCB + c;
    live[c] = idx[c] < n;
    fixT[c] = fixT_all != 0;
    if (live[c] && ty) {
      const int k = idx[c], tt = ty[k];
      if (tt == EMPTY) live[c] = false;
      else if (bc_proc(tt) && !sprim[k]) {   // processor [internal n] slot: copy the cell's values
        const int cc = bfc[k];
        if (l == 0) { T[k] = cT[cc]; he[k] = che[cc]; psi[k] = cpsi[cc]; rho[k] = crho[cc]; mu[k] = cmu[cc]; alpha[k] = calpha[cc]; }
        for (int i = l; i < S; i += TG) { rhoD[(long)i * n + k] = crhoD[i * Cc + cc]; hai[(long)i * n + k] = chai[i * Cc + cc]; }
        live[c] = false;
      } else if (bc_fixes_value(tt)) fixT[c] = true;
    }
    if (!live[c]) fixT[c] = true;
    if (l == 0) sLive[grp * NCB + c] = live[c];
  }
  // species owned by this lane; cells without work evaluate a dummy state (uniform barriers below)
  double X[NCB][SPL], ryw[NCB][SPL], Wm[NCB];
#pragma unroll
  for (int c = 0; c < NCB; ++c) {
    double y[SPL], sum = 0.0;
#pragma unroll
    for (int q = 0; q < SPL; ++q) {
      const int i = q * TG + l;
      y[q] = (i < S) ? (live[c] ? sX[grp * NCB + c][i] : (i == 0 ? 1.0 : 0.0)) : 0.0;
      if (i < S) sum += y[q] * t.rW[i];
    }
    const double rsum = 1.0 / gsum<TG>(sum);
    double wm = 0.0;
#pragma unroll
    for (int q = 0; q < SPL; ++q) {
      const int i = q * TG + l;
      X[c][q] = i < S ? y[q] * t.rW[i] * rsum : 0.0;
      ryw[c][q] = i < S ? R_GAS * t.rW[i] * y[q] : 0.0;
      if (i < S) wm += X[c][q] * t.W[i];
    }
    Wm[c] = gsum<TG>(wm);
  }
  double Tc[NCB], hc[NCB], pc[NCB];
#pragma unroll
  for (int c = 0; c < NCB; ++c) {
    Tc[c] = live[c] ? T[idx[c]] : 300.0;
    hc[c] = live[c] ? he[idx[c]] : 0.0;
    pc[c] = live[c] ? p[idx[c]] : 101325.0;
  }
  // the lane's NASA coefficients, both ranges, loaded once for the Newton loop, the final h / cp and h_i
  double nhi[SPL][6], nlo[SPL][6], ntm[SPL];
#pragma unroll
  for (int q = 0; q < SPL; ++q) {
    const int i = q * TG + l;
    const double* a = t.nasaT + (i < S ? i : 0);
    ntm[q] = a[0];
#pragma unroll
    for (int k = 0; k < 6; ++k) { nhi[q][k] = a[(1 + k) * S]; nlo[q][k] = a[(8 + k) * S]; }
  }
  // mixture h and cp of the cells flagged in `on` at temperatures TT (each cell picks its range)
  auto hcp = [&](const double (&TT)[NCB], const bool (&on)[NCB], double (&h)[NCB], double (&cp)[NCB]) {
    double hh[NCB], cc[NCB];
    double P1[NCB], P2[NCB], P3[NCB], P4[NCB], Q1[NCB], Q2[NCB], Q3[NCB], Q4[NCB], RT[NCB];
#pragma unroll
    for (int c = 0; c < NCB; ++c) {
      hh[c] = 0.0; cc[c] = 0.0;
      const double T1 = TT[c], T2 = T1 * T1, T3 = T2 * T1, T4 = T3 * T1;
      P1[c] = T1; P2[c] = T2; P3[c] = T3; P4[c] = T4;
      Q1[c] = T1 * 0.5; Q2[c] = T2 * (1.0 / 3.0); Q3[c] = T3 * 0.25; Q4[c] = T4 * (1.0 / 5.0); RT[c] = rcp_nr(T1);
    }
#pragma unroll
    for (int q = 0; q < SPL; ++q) {
      const int i = q * TG + l;
      if (i < S) {
        const double tm = ntm[q];
        const double (&hi)[6] = nhi[q];
        const double (&lo)[6] = nlo[q];
#pragma unroll
        for (int c = 0; c < NCB; ++c) {
          const double T1 = TT[c];
          const bool up = T1 > tm;
          const double a0 = up ? hi[0] : lo[0], a1 = up ? hi[1] : lo[1], a2 = up ? hi[2] : lo[2];
          const double a3 = up ? hi[3] : lo[3], a4 = up ? hi[4] : lo[4], a5 = up ? hi[5] : lo[5];
          const double c1 = a0 + a1 * P1[c] + a2 * P2[c] + a3 * P3[c] + a4 * P4[c];
          const double h1 = a0 + a1 * Q1[c] + a2 * Q2[c] + a3 * Q3[c] + a4 * Q4[c] + a5 * RT[c];
          hh[c] += h1 * T1 * ryw[c][q];
          cc[c] += c1 * ryw[c][q];
        }
      }
    }
#pragma unroll
    for (int c = 0; c < NCB; ++c)
      if (on[c]) { h[c] = gsum<TG>(hh[c]); cp[c] = gsum<TG>(cc[c]); }
  };
  double cpm[NCB];
  {
    bool act[NCB], any = false;
#pragma unroll
    for (int c = 0; c < NCB; ++c) { act[c] = !fixT[c]; any = any || act[c]; }
    for (int it = 0; it < 20 && any; ++it) {
      double h[NCB], cp[NCB];
      hcp(Tc, act, h, cp);
      any = false;
#pragma unroll
      for (int c = 0; c < NCB; ++c)
        if (act[c]) {
          const double dT = (h[c] - hc[c]) / cp[c];
          Tc[c] -= dT;
          if (fabs(h[c] - hc[c]) < 1e-7 || fabs(dT / Tc[c]) < 1e-7) act[c] = false;
          any = any || act[c];
        }
    }
    bool all[NCB];
    double h[NCB];
#pragma unroll
    for (int c = 0; c < NCB; ++c) { all[c] = true; h[c] = 0.0; }
    hcp(Tc, all, h, cpm);
#pragma unroll
    for (int c = 0; c < NCB; ++c)
      if (fixT[c]) hc[c] = h[c];
  }
  // from here on each result is stored as soon as it is known (short live ranges: NCB cells' state
  // stays in registers without spilling)
  double poly[NCB][5], sT[NCB], rdp[NCB];
#pragma unroll
  for (int c = 0; c < NCB; ++c) {
    const double lnT = log(Tc[c]);
    poly[c][0] = 1.0; poly[c][1] = lnT; poly[c][2] = lnT * lnT; poly[c][3] = lnT * poly[c][2];
    poly[c][4] = poly[c][2] * poly[c][2];
    sT[c] = sqrt(Tc[c]);
    const double ps = Wm[c] / (R_GAS * Tc[c]), rh = pc[c] * ps;
    rdp[c] = rh / pc[c];
    if (live[c] && l == 0) { const int k = idx[c]; T[k] = Tc[c]; he[k] = hc[c]; psi[k] = ps; rho[k] = rh; }
  }
  // species enthalpies hai (depend on T only)
  double ha[NCB][SPL];
#pragma unroll
  for (int q = 0; q < SPL; ++q) {
    const int i = q * TG + l;
#pragma unroll
    for (int c = 0; c < NCB; ++c) ha[c][q] = 0.0;
    if (i >= S) continue;
    const double tm = ntm[q], rw = R_GAS * t.rW[i];
#pragma unroll
    for (int c = 0; c < NCB; ++c) {
      const double T1 = Tc[c], T2 = T1 * T1, T3 = T2 * T1, T4 = T3 * T1;
      const bool up = T1 > tm;
      double a[6];
#pragma unroll
      for (int k = 0; k < 6; ++k) a[k] = up ? nhi[q][k] : nlo[q][k];
      const double h1 = a[0] + a[1] * (T1 * 0.5) + a[2] * (T2 * (1.0 / 3.0)) +
                        a[3] * (T3 * 0.25) + a[4] * (T4 * (1.0 / 5.0)) + a[5] * rcp_nr(T1);
      ha[c][q] = h1 * T1 * rw;
    }
  }
  {
    double sv[NCB][SPL];
#pragma unroll
    for (int q = 0; q < SPL; ++q) {
      const int i = q * TG + l;
      double vc[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) vc[k] = i < S ? t.visc[i * 5 + k] : 0.0;
#pragma unroll
      for (int c = 0; c < NCB; ++c) {
        double dp = 0.0;
#pragma unroll
        for (int k = 0; k < 5; ++k) dp += vc[k] * poly[c][k];
        sv[c][q] = dp;
        sP[grp * NCB + c][i] = make_double2(X[c][q] * (1.0 / SQRT8), rcp_nr(dp));   // lanes past S: unused entries
      }
    }
    group_sync<TG>();
    // Wilke rows
    double mpart[NCB];
#pragma unroll
    for (int c = 0; c < NCB; ++c) mpart[c] = 0.0;
#pragma unroll
    for (int q = 0; q < SPL; ++q) {
      const int i = q * TG + l;
      if (i >= S) break;
      double s2[NCB];
#pragma unroll
      for (int c = 0; c < NCB; ++c) s2[c] = 0.0;
#pragma unroll 4
      for (int j = 0; j < S; ++j) {
        const double2 vp = vcP[j * S + i];   // {vc1, vc2}: one 16-B load
        const double v1 = vp.x, v2 = vp.y;
#pragma unroll
        for (int c = 0; c < NCB; ++c) {
          const double2 xr = sP[grp * NCB + c][j];
          const double tmp = 1.0 + (sv[c][q] * xr.y) * v2;
          s2[c] += xr.x * v1 * (tmp * tmp);
        }
      }
#pragma unroll
      for (int c = 0; c < NCB; ++c) mpart[c] += X[c][q] * (sv[c][q] * sv[c][q]) * rcp_nr(s2[c]);
    }
#pragma unroll
    for (int c = 0; c < NCB; ++c) {
      const double mum = gsum<TG>(mpart[c]) * sT[c];
      if (live[c] && l == 0) mu[idx[c]] = mum;
    }
  }
  {
    double sc[NCB], sic[NCB];
#pragma unroll
    for (int c = 0; c < NCB; ++c) { sc[c] = 0.0; sic[c] = 0.0; }
#pragma unroll
    for (int q = 0; q < SPL; ++q) {
      const int i = q * TG + l;
      if (i >= S) break;
      double kc[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) kc[k] = t.cond[i * 5 + k];
#pragma unroll
      for (int c = 0; c < NCB; ++c) {
        double dp = 0.0;
#pragma unroll
        for (int k = 0; k < 5; ++k) dp += kc[k] * poly[c][k];
        const double lam = dp * sT[c];
        sc[c] += X[c][q] * lam;
        sic[c] += X[c][q] * rcp_nr(lam);
      }
    }
#pragma unroll
    for (int c = 0; c < NCB; ++c) {
      const double al = 0.5 * (gsum<TG>(sc[c]) + 1.0 / gsum<TG>(sic[c])) / cpm[c];
      if (live[c] && l == 0) alpha[idx[c]] = al;
    }
  }
  group_sync<TG>();   // mole fractions (unscaled) for the diffusion rows
#pragma unroll
  for (int q = 0; q < SPL; ++q) {
    const int i = q * TG + l;
#pragma unroll
    for (int c = 0; c < NCB; ++c) {
      sX[grp * NCB + c][i] = X[c][q];
      sP[grp * NCB + c][i] = make_double2(X[c][q], X[c][q] * t.W[i < S ? i : 0]);   // {x_j, x_j W_j}
    }
  }
  group_sync<TG>();
  double rpT[NCB], rdv[NCB][SPL];
#pragma unroll
  for (int c = 0; c < NCB; ++c) rpT[c] = 1.0 / (Tc[c] * sT[c]);
  if (SPL == 1 && t.bdR) {
    // symmetric fits, one species per lane: each unordered pair is evaluated once. At rotation step d lane i
    // evaluates 1 / D of the pair (i, i + d mod S) and receives from lane i - d that of (i - d, i): d = 1 .. S / 2
    // covers every pair of an odd S once; for an even S the pair (i, i + S / 2) of the last step is evaluated by
    // both its lanes and each keeps its own value. Half the fit evaluations, reciprocals and coefficient loads of
    // the row loop below; the row sums are accumulated in rotation order (agrees to rounding).
    const int i = l;
    double s1[NCB], s2[NCB];
#pragma unroll
    for (int c = 0; c < NCB; ++c) { s1[c] = 0.0; s2[c] = 0.0; }
    const int D = S / 2;
    const int gb = threadIdx.x - l;   // the group's lane 0
#pragma unroll 2
    for (int d = 1; d <= D; ++d) {
      const int jp = i + d < S ? i + d : i + d - S, jm = i - d >= 0 ? i - d : i - d + S;
      const bool own = i < S;
      const int e = (d - 1) * S + (own ? i : 0);
      const double2 b01 = bdp[e], b23 = bdp[DS + e], b4p = bdp[2 * DS + e];
      const bool both = 2 * d != S;   // the received value is a different pair's
#pragma unroll
      for (int c = 0; c < NCB; ++c) {
        const double tmp = b01.x * poly[c][0] + b01.y * poly[c][1] + b23.x * poly[c][2] + b23.y * poly[c][3] +
                           b4p.x * poly[c][4];
        const double inv = rcp_nr(tmp);   // T^1.5 / D_ij: the common factor 1 / T^1.5 applied to the row sums
        const double inr = __shfl(inv, gb + (own ? jm : 0), 64);
        // lanes past S accumulate in-bounds garbage (their rows and their 1/D are never used): no branch
        const double2 xp = sP[grp * NCB + c][jp], xm = sP[grp * NCB + c][jm];
        s1[c] += xp.x * inv;
        s2[c] += xp.y * inv;
        if (both) { s1[c] += xm.x * inr; s2[c] += xm.y * inr; }
      }
    }
#pragma unroll
    for (int c = 0; c < NCB; ++c) {
      s1[c] *= rpT[c];
      s2[c] *= rpT[c];
      double rd = 0.0;
      if (i < S && !(X[c][0] + 1e-10 > 1.)) {
        const double q2 = s2[c] * (X[c][0] * rcp_nr(Wm[c] - X[c][0] * t.W[i]));
        rd = rcp_nr(s1[c] + q2) * rdp[c];
      }
      rdv[c][0] = rd;
    }
  } else
#pragma unroll
  for (int q = 0; q < SPL; ++q) {
    const int i = q * TG + l;
    if (i >= S) break;
    double s1[NCB], s2[NCB];
#pragma unroll
    for (int c = 0; c < NCB; ++c) { s1[c] = 0.0; s2[c] = 0.0; }
    for (int j = 0; j < S; ++j) {
      const double* bd = t.bdiffT + j * 5 * S + i;
      const double b0 = bd[0], b1 = bd[S], b2 = bd[2 * S], b3 = bd[3 * S], b4 = bd[4 * S];
      const double wj = t.W[j];
#pragma unroll
      for (int c = 0; c < NCB; ++c) {
        const double tmp = b0 * poly[c][0] + b1 * poly[c][1] + b2 * poly[c][2] + b3 * poly[c][3] + b4 * poly[c][4];
        const double inv = rpT[c] * rcp_nr(tmp);    // 1 / D_ij, D_ij = T^1.5 poly(ln T)
        const double xj = j == i ? 0.0 : sX[grp * NCB + c][j];
        s1[c] += xj * inv;
        s2[c] += xj * wj * inv;
      }
    }
#pragma unroll
    for (int c = 0; c < NCB; ++c) {
      double rd = 0.0;
      if (!(X[c][q] + 1e-10 > 1.)) {
        const double q2 = s2[c] * (X[c][q] * rcp_nr(Wm[c] - X[c][q] * t.W[i]));
        rd = rcp_nr(s1[c] + q2) * rdp[c];
      }
      rdv[c][q] = rd;
    }
  }
#pragma unroll
  for (int q = 0; q < SPL; ++q) {   // the group's own rows (read only by this group, all reads done)
    const int i = q * TG + l;
#pragma unroll
    for (int c = 0; c < NCB; ++c)
      sX[grp * NCB + c][i] = rdv[c][q], sR[grp * NCB + c][i] = ha[c][q];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < CPB * S; e += TCB) {
    const int sp = e / CPB, cl = e % CPB;
    if (base + cl < n && sLive[cl]) {
      rhoD[(long)sp * n + base + cl] = sX[cl][sp];
      hai[(long)sp * n + base + cl] = sR[cl][sp];
    }
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

// hc_i = Hf298SS_i / W_i [J/kg] (dfChemistryModel.C:335-338): Cantera's NasaPoly2::reportHf298 -- the NASA7 range
// holding 298.15 K (the low one when 298.15 <= T_mid), h/RT by NasaPoly1::updateProperties' expression
// (ct_k = a_k T^k; h/RT = ct0 + ct1/2 + ct2/3 + ct3/4 + ct4/5 + a5/T), times GasConstant * 298.15.
// oracle/chem_oracle.py:hf298_per_mass restates the same expression in the same order.
std::vector<double> heat_of_formation_per_mass(int S, const double* W, const double* nasa) {
  std::vector<double> hc(S);
  const double T = 298.15, T2 = T * T, T3 = T2 * T, T4 = T3 * T, rT = 1.0 / T;
  for (int i = 0; i < S; ++i) {
    const double* row = nasa + 15 * i;
    const double* a = T <= row[0] ? row + 8 : row + 1;
    const double ct0 = a[0], ct1 = a[1] * T, ct2 = a[2] * T2, ct3 = a[3] * T3, ct4 = a[4] * T4;
    const double h_RT = ct0 + 0.5 * ct1 + (1.0 / 3.0) * ct2 + 0.25 * ct3 + 0.2 * ct4 + a[5] * rT;
    hc[i] = h_RT * R_GAS * T / W[i];
  }
  return hc;
}

void thermo_upload(Ctx& x) {
  Thermo& t = x.thermo;
  t.dW.upload(t.W, x.stream);
  {
    std::vector<double> rw(t.W.size());
    for (size_t i = 0; i < rw.size(); ++i) rw[i] = 1.0 / t.W[i];
    t.drW.upload(rw, x.stream);
    DFMI_HIP(hipStreamSynchronize(x.stream));
  }
  t.dnasa.upload(t.nasa, x.stream);
  t.hc = heat_of_formation_per_mass(t.S, t.W.data(), t.nasa.data());
  t.dhc.upload(t.hc, x.stream);
  t.dvisc.upload(t.visc, x.stream);
  t.dcond.upload(t.cond, x.stream);
  t.dbdiff.upload(t.bdiff, x.stream);
  t.dvc1.upload(t.vc1, x.stream);
  t.dvc2.upload(t.vc2, x.stream);
  const int S = t.S;
  std::vector<double> nT(15 * S), bT(5 * S * S), v1(S * S), v2(S * S);
  for (int i = 0; i < S; ++i) {
    for (int k = 0; k < 15; ++k) nT[k * S + i] = t.nasa[i * 15 + k];
    for (int j = 0; j < S; ++j) {
      for (int k = 0; k < 5; ++k) bT[(j * 5 + k) * S + i] = t.bdiff[(i * S + j) * 5 + k];
      v1[j * S + i] = t.vc1[i * S + j];
      v2[j * S + i] = t.vc2[i * S + j];
    }
  }
  t.dnasaT.upload(nT, x.stream);
  t.dbdiffT.upload(bT, x.stream);
  t.dvc1T.upload(v1, x.stream);
  t.dvc2T.upload(v2, x.stream);
  std::vector<double> vp(2 * S * S), br;
  for (int j = 0; j < S; ++j)
    for (int i = 0; i < S; ++i) { vp[(j * S + i) * 2] = t.vc1[i * S + j]; vp[(j * S + i) * 2 + 1] = t.vc2[i * S + j]; }
  t.dvcP.upload(vp, x.stream);
  bool sym = true;
  for (int i = 0; i < S && sym; ++i)
    for (int j = 0; j < S && sym; ++j)
      for (int k = 0; k < 5; ++k)
        if (t.bdiff[(i * S + j) * 5 + k] != t.bdiff[(j * S + i) * 5 + k]) { sym = false; break; }
  if (sym && S > 1) {
    const int D = S / 2;
    // three planes of D * S pairs {b0, b1}, {b2, b3}, {b4, 0}: lane i's pair (i, i + d) at (d - 1) * S + i
    const size_t DS = (size_t)D * S;
    br.assign(DS * 6, 0.0);
    for (int d = 1; d <= D; ++d)
      for (int i = 0; i < S; ++i)
        for (int k = 0; k < 5; ++k)
          br[((k / 2) * DS + (size_t)(d - 1) * S + i) * 2 + k % 2] = t.bdiff[(i * S + (i + d) % S) * 5 + k];
    t.dbdR.upload(br, x.stream);
  } else {
    t.dbdR.release();
  }
  DFMI_HIP(hipStreamSynchronize(x.stream));   // the staging vectors above go out of scope
}

void thermo_energy_gradient(Ctx& x) {
  Thermo& th = x.thermo;
  DFMI_CHECK(th.S == x.S, "thermo coefficients not set or species count mismatch");
  if (x.B == 0) return;
  const auto& pt = x.pt("he");
  bool any = false;
  for (int p = 0; p < x.P; ++p) any = any || pt[p] == GRADIENT_ENERGY;
  if (!any) return;   // the field stays zero
  TC t{th.dW, th.drW, th.dnasa, th.dvisc, th.dcond, th.dbdiff, th.dvc1, th.dvc2, 0, th.dnasaT, th.dbdiffT, th.dvc1T, th.dvc2T,
       th.dvcP, nullptr};
  MeshView m = x.view();
#define CALL(NS)                                                                                                  \
  hipLaunchKernelGGL(k_energy_gradient<NS>, dim3(blocks_for(x.B, 256)), dim3(256), 0, x.stream, m, t, x.st("he"), \
                     x.f("T"), x.f("Y"), x.f("boundary_Y"), x.f("boundary_heGradient"))
  if (species_generic(x))
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

void thermo_correct(Ctx& x, bool from_T, int part) {
  Thermo& th = x.thermo;
  DFMI_CHECK(part >= TH_ALL && part <= TH_TRANSPORT, "thermo_correct: part 0, 1 or 2");
  // the species-generic (cooperative) kernel is not split: its TH_STATE call does the whole update
  if (species_generic(x) && part == TH_TRANSPORT) return;
  DFMI_CHECK(th.S == x.S, "thermo coefficients not set or species count mismatch");
  int sym = 1;
  for (int i = 0; i < th.S && sym; ++i)
    for (int j = 0; j < th.S && sym; ++j)
      for (int k = 0; k < 5; ++k)
        if (th.bdiff[(i * th.S + j) * 5 + k] != th.bdiff[(j * th.S + i) * 5 + k]) { sym = 0; break; }
  TC t{th.dW, th.drW, th.dnasa, th.dvisc, th.dcond, th.dbdiff, th.dvc1, th.dvc2, sym, th.dnasaT, th.dbdiffT, th.dvc1T, th.dvc2T,
       th.dvcP, sym && th.dbdR.n ? th.dbdR.p : nullptr};
  MeshView m = x.view();
#define CALL(NS) do { switch (part) { case TH_ALL: CALLP(NS, TH_ALL); break;                                  \
    case TH_STATE: CALLP(NS, TH_STATE); break; default: CALLP(NS, TH_TRANSPORT); } } while (0)
  static const char* kname[3] = {"k_thermo_cells", "k_thermo_state", "k_thermo_transport"};
#define CALLP(NS, PART)                                                                                           \
  do {                                                                                                            \
    if (x.C > 0) { KScope _ks(x, kname[PART]);                                                                    \
      hipLaunchKernelGGL((k_thermo_cells<NS, PART>), dim3(blocks_for(x.C, 256)), dim3(256), 0, x.stream, x.C, t,    \
                         (int)from_T, x.f("T"), x.f("he"), x.f("p"), x.f("Y"), x.f("psi"), x.f("rho"), x.f("mu"),   \
                         x.f("alpha"), x.f("rhoD"), x.f("hai")); }                                              \
    DFMI_HIP(hipGetLastError());                                                                                  \
    if (x.B > 0) hipLaunchKernelGGL((k_thermo_slots<NS, PART>), dim3(blocks_for(x.B, 256)), dim3(256), 0, x.stream, m, t,\
                       x.st("T"), (int)from_T, x.f("T"), x.f("he"), x.f("psi"), x.f("rho"), x.f("mu"), x.f("alpha"), \
                       x.f("rhoD"), x.f("hai"), x.f("boundary_T"), x.f("boundary_he"), x.f("boundary_p"),          \
                       x.f("boundary_Y"), x.f("boundary_psi"), x.f("boundary_rho"), x.f("boundary_mu"),            \
                       x.f("boundary_alpha"), x.f("boundary_rhoD"), x.f("boundary_hai"));                         \
    DFMI_HIP(hipGetLastError());                                                                                  \
  } while (0)
  if (species_generic(x)) {
    DFMI_CHECK(x.S <= SMAX, "thermo: at most 64 species");
    // 64 lanes per cell group, 4 cells per group (TG x NCB = 16x1 / 16x2 / 16x4 / 64x2 / 64x4 / 64x8 measured
    // 26 / 14.6 / 16.5 / 16.3 / 13.7 / 21.4 ms per call on 2M cells x 53 species)
#define COOP(TG, NCB)                                                                                                  \
  do {                                                                                                            \
    constexpr int CPB = TCB / TG * NCB;                                                                           \
    if (x.C > 0) {                                                                                                \
      KScope _ks(x, "k_thermo_cells");                                                                            \
      hipLaunchKernelGGL((k_thermo_coop<TG, NCB>), dim3(blocks_for(x.C, CPB)), dim3(TCB), 0, x.stream, x.C, x.S, t,     \
                         (int)from_T, (const int8_t*)nullptr, (const int8_t*)nullptr, (const int*)nullptr, 0L,    \
                         (const double*)nullptr, (const double*)nullptr, (const double*)nullptr,                 \
                         (const double*)nullptr, (const double*)nullptr, (const double*)nullptr,                 \
                         (const double*)nullptr, (const double*)nullptr, x.f("T"), x.f("he"), x.f("p"), x.f("Y"), \
                         x.f("psi"), x.f("rho"), x.f("mu"), x.f("alpha"), x.f("rhoD"), x.f("hai"));              \
    }                                                                                                             \
    DFMI_HIP(hipGetLastError());                                                                                  \
    if (x.B > 0)                                                                                                  \
      hipLaunchKernelGGL((k_thermo_coop<TG, NCB>), dim3(blocks_for(x.B, CPB)), dim3(TCB), 0, x.stream, x.B, x.S, t,     \
                         (int)from_T, x.st("T"), m.sprim, m.bfc, (long)x.C, x.f("T"), x.f("he"), x.f("psi"),      \
                         x.f("rho"), x.f("mu"), x.f("alpha"), x.f("rhoD"), x.f("hai"), x.f("boundary_T"),         \
                         x.f("boundary_he"), x.f("boundary_p"), x.f("boundary_Y"), x.f("boundary_psi"),           \
                         x.f("boundary_rho"), x.f("boundary_mu"), x.f("boundary_alpha"), x.f("boundary_rhoD"),    \
                         x.f("boundary_hai"));                                                                    \
    DFMI_HIP(hipGetLastError());                                                                                  \
  } while (0)
    COOP(64, 4);
#undef COOP
  } else switch (x.S) {
    case 2: CALL(2); break; case 3: CALL(3); break; case 4: CALL(4); break; case 5: CALL(5); break;
    case 6: CALL(6); break; case 7: CALL(7); break; case 8: CALL(8); break; case 9: CALL(9); break;
    case 10: CALL(10); break; case 11: CALL(11); break; case 12: CALL(12); break; case 13: CALL(13); break;
    case 14: CALL(14); break; case 15: CALL(15); break; case 16: CALL(16); break;
    default: throw Error("dfmi: thermo species count " + std::to_string(x.S) + " not supported");
  }
#undef CALL
#undef CALLP
  // neighbour halves of the processor slots carry the neighbour rank's cell values
  if (species_generic(x)) part = TH_ALL;
  std::vector<const char*> names;
  if (from_T && part != TH_TRANSPORT) names.push_back("he");
  if (part != TH_TRANSPORT) for (const char* f : {"T", "psi", "rho"}) names.push_back(f);
  if (part != TH_STATE) for (const char* f : {"mu", "alpha", "rhoD", "hai"}) names.push_back(f);
  halo_fields(x, names);
}

}  // namespace dfmi
