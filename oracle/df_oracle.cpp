// df_oracle.cpp -- CPU restatement of the dfLowMachFoam GPU hot path (TEST INFRASTRUCTURE).
//
// ORACLE HEADER: this file is the parity checker, not the product. Only tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it. It restates,
// in OpenFOAM's sequential face-loop form, what the reference GPU path
// (show-me-code/deepflame-dev src_gpu/*.cu, driven by
// applications/solvers/dfLowMachFoam/*_GPU.H) computes, with the CPU-dfLowMachFoam
// semantics fixes listed in DESIGN.md "Deviations" (SURVEY.md Appendix A). Every
// routine cites the reference file:line it follows.
//
// Parity status: the reference (OpenFOAM-7 + Cantera-2.6 + CUDA + AmgX) cannot be
// built or run here. Thermo/transport is pinned by the reference's own
// fixture thermo_ES80_H2-7-16.txt (tests/golden); the finite-volume part is pinned by
// analytic invariants only (exact Gauss gradients of linear fields, discrete
// conservation, symmetric laplacian): "parity unpinned" against reference outputs.
//
// Canonical arithmetic (what the HIP kernels reproduce bit-for-bit):
//  * every fvm/fvc term is its own partial sum, exactly as OpenFOAM builds one
//    fvMatrix per term: start from 0, visit internal faces in increasing face index
//    (owner +=, neighbour -=, lduMatrix::negSumDiag / fvc::surfaceIntegrate), then
//    boundary slots in increasing slot order; terms are then combined in the order
//    of the C++ expression in *Eqn.H (fvMatrix operator+/-/==);
//  * face formulas are OpenFOAM's (gaussConvectionScheme::fvmDiv, gaussLaplacianScheme,
//    surfaceInterpolation linear weights); explicit fvc terms enter the source as the
//    face sum itself (the reference skips the /V then *V round trip);
//  * built with -ffp-contract=off (the reference used -fmad=false, src_gpu/CMakeLists.txt:17).
//
// Parallelism (OpenMP): the per-face scatter "owner +=, neighbour -=" is evaluated as a per-cell
// gather over the cell's faces in increasing face index -- the very order in which the sequential
// loop would have added them -- so every partial sum is bitwise the sequential one. Boundary-slot
// scatters stay sequential (several slots may share a cell).
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>
#include <stdexcept>
#include <algorithm>

namespace {

enum BC { ZG = 0, FV = 1, COUPLED = 2, EMPTY = 3, GRAD_E = 4, CALC = 5, CYCLIC = 6, PROC = 7, EXTRAP = 8,
          FIX_E = 9, PROC_CYC = 10, WAVE = 11, IN_OUT = 12 };
// mixedFvPatchField family: waveTransmissive (advectiveFvPatchField, OpenFOAM-7; the 1D flame's outlet p,
// test/Tu500K-Phi1/0/p:34) and inletOutlet; value = f ref + (1 - f) cell
inline bool is_mixed(int t) { return t == WAVE || t == IN_OUT; }
inline bool is_coupled(int t) { return t == CYCLIC || t == PROC || t == PROC_CYC || t == COUPLED; }
inline bool is_proc(int t) { return t == PROC || t == PROC_CYC; }
inline bool fixes_value(int t) { return t == FV || t == FIX_E; }

std::map<std::string, double*> D;
std::map<std::string, int*> I;
std::string g_err;

double* d(const char* k) {
  auto it = D.find(k);
  if (it == D.end()) throw std::runtime_error(std::string("oracle: missing double array ") + k);
  return it->second;
}
bool has(const char* k) { return D.count(k) != 0; }
int* ia(const char* k) {
  auto it = I.find(k);
  if (it == I.end()) throw std::runtime_error(std::string("oracle: missing int array ") + k);
  return it->second;
}

// cell -> faces, merged in increasing face index: entry f (cell owns f) or ~f (cell is f's neighbour)
struct CellFaces {
  const int *own = nullptr, *nei = nullptr;
  int C = -1, F = -1;
  std::vector<int> start, face;
};
CellFaces g_cf;
const CellFaces& cell_faces(int C, int F, const int* own, const int* nei) {
  if (g_cf.own == own && g_cf.nei == nei && g_cf.C == C && g_cf.F == F) return g_cf;
  g_cf.own = own; g_cf.nei = nei; g_cf.C = C; g_cf.F = F;
  g_cf.start.assign(C + 1, 0);
  for (int f = 0; f < F; ++f) { g_cf.start[own[f] + 1]++; g_cf.start[nei[f] + 1]++; }
  for (int c = 0; c < C; ++c) g_cf.start[c + 1] += g_cf.start[c];
  g_cf.face.resize(2L * F);
  std::vector<int> pos(g_cf.start.begin(), g_cf.start.end() - 1);
  for (int f = 0; f < F; ++f) { g_cf.face[pos[own[f]]++] = f; g_cf.face[pos[nei[f]]++] = ~f; }   // f ascending
  return g_cf;
}

struct M {
  int C, F, B, P, S;
  const int *own, *nei, *psize, *cyc_nbr, *bfc, *kind;
  const double *Sf, *magSf, *w, *dc, *V, *bSf, *bmagSf, *bw, *bdc;
  std::vector<int> poff, slot_patch, primary, partner_cell;
  const int *cfs, *cff;   // cell_faces
  double rdt;
  double sf(int k, int f) const { return Sf[(long)k * F + f]; }
  double bsf(int k, int b) const { return bSf[(long)k * B + b]; }
};

M mesh() {
  M m;
  int* dims = ia("dims");
  m.C = dims[0]; m.F = dims[1]; m.B = dims[2]; m.P = dims[3]; m.S = dims[4];
  m.own = ia("owner"); m.nei = ia("neighbour"); m.psize = ia("patch_size");
  m.cyc_nbr = ia("cyclic_neighbor"); m.bfc = ia("boundary_face_cell"); m.kind = ia("patch_kind");
  m.Sf = d("sf"); m.magSf = d("mag_sf"); m.w = d("weight"); m.dc = d("delta_coeffs"); m.V = d("volume");
  m.bSf = d("boundary_sf"); m.bmagSf = d("boundary_mag_sf"); m.bw = d("boundary_weight");
  m.bdc = d("boundary_delta_coeffs");
  m.rdt = d("rdelta_t")[0];
  const CellFaces& cf = cell_faces(m.C, m.F, m.own, m.nei);
  m.cfs = cf.start.data(); m.cff = cf.face.data();
  m.poff.resize(m.P + 1);
  m.slot_patch.assign(m.B, -1);
  m.primary.assign(m.B, 0);
  m.partner_cell.assign(m.B, -1);
  int off = 0;
  for (int p = 0; p < m.P; ++p) {
    m.poff[p] = off;
    int n = m.psize[p];
    int slots = (m.kind[p] == 2) ? 2 * n : n;
    for (int i = 0; i < slots; ++i) { m.slot_patch[off + i] = p; m.primary[off + i] = (i < n); }
    off += slots;
  }
  m.poff[m.P] = off;
  if (off != m.B) throw std::runtime_error("oracle: boundary slot count mismatch");
  for (int p = 0; p < m.P; ++p)
    if (m.kind[p] == 1)
      for (int i = 0; i < m.psize[p]; ++i) m.partner_cell[m.poff[p] + i] = m.bfc[m.poff[m.cyc_nbr[p]] + i];
  return m;
}

// Neighbour-side cell value of a coupled slot: cyclic -> partner face's cell; processor ->
// the received neighbour value held in the slot ([neighbour n | internal n], createGPUSolver.H:265-304).
inline double nbr(const M& m, const double* vf, const double* bvf, int b) {
  return m.partner_cell[b] >= 0 ? vf[m.partner_cell[b]] : bvf[b];
}
inline double interp_f(double w, double vo, double vn) { return w * (vo - vn) + vn; }      // surfaceInterpolation::interpolate
inline double interp_b(double w, double vo, double vn) { return w * vo + (1.0 - w) * vn; } // coupledFvPatchField::evaluate

// per-slot data of a field's mixed conditions: waveTransmissive valueFraction (set at the pEqn
// assembly) and refValue = old-time boundary value; inletOutlet valueFraction = 1 - pos0(phi_b),
// refValue = inletValue
struct Mix { const double *wvf, *wref, *bphi, *ioref; };
Mix mix_for(const std::string& field) {
  Mix x{nullptr, nullptr, nullptr, nullptr};
  if (has("boundary_phi")) x.bphi = d("boundary_phi");
  if (field == "p" && has("boundary_p_vf")) { x.wvf = d("boundary_p_vf"); x.wref = d("boundary_p_old"); }
  std::string r = "boundary_" + field + "_ref";
  if (has(r.c_str())) x.ioref = d(r.c_str());
  return x;
}
inline void mix_vf_ref(int t, const Mix& x, int b, int B, int comp, double& vf, double& ref) {
  if (t == WAVE) { vf = x.wvf[b]; ref = x.wref[b]; }
  else { vf = x.bphi[b] >= 0.0 ? 0.0 : 1.0; ref = x.ioref[(long)comp * B + b]; }
}

// value/gradient coefficients (valueInternalCoeffs etc.; dfMatrixOpBase.cu:279-621)
struct BCoef { double vic, vbc, gic, gbc; };
inline BCoef bcoef(int t, double bval, double w, double bdc, double egrad = 0.0) {
  switch (t) {
    case ZG: case EXTRAP: return {1., 0., 0., 0.};
    case FV: case FIX_E: return {0., bval, -1 * bdc, bdc * bval};
    case GRAD_E: return {1., egrad / bdc, 0., egrad};
    default: return {w, 1.0 - w, -1 * bdc, bdc};   // coupled
  }
}

// the same, for a field that may carry mixed conditions (mixedFvPatchField::value/gradient*Coeffs)
inline BCoef bcoef_f(int t, double bval, double w, double bdc, const Mix& mx, int b, int B, int comp, double egrad = 0.0) {
  if (is_mixed(t)) {
    double vf, ref;
    mix_vf_ref(t, mx, b, B, comp, vf, ref);
    return {1.0 - vf, vf * ref, -vf * bdc, vf * bdc * ref};
  }
  return bcoef(t, bval, w, bdc, egrad);
}

template <class FN> void for_slots(const M& m, const int* type, FN fn) {
  for (int b = 0; b < m.B; ++b) {
    if (!m.primary[b]) continue;
    int t = type[m.slot_patch[b]];
    if (t == EMPTY) continue;
    fn(b, t, m.bfc[b]);
  }
}

// per-cell gather of face terms in increasing face index: fo(f) where the cell owns f, fn(f) where
// it is f's neighbour, folded into a sum starting from 0
template <class FO, class FN> void gather(const M& m, double* s, FO fo, FN fn) {
#pragma omp parallel for schedule(static)
  for (int c = 0; c < m.C; ++c) {
    double a = 0.0;
    for (int e = m.cfs[c]; e < m.cfs[c + 1]; ++e) {
      const int f = m.cff[e];
      a = f >= 0 ? fo(a, f) : fn(a, ~f);
    }
    s[c] = a;
  }
}
// fvc::surfaceIntegrate without the /V: owner +=, neighbour -=, then boundary +=
template <class FF, class FB> std::vector<double> integrate(const M& m, const int* type, FF face, FB bnd) {
  std::vector<double> v(m.F), s(m.C);
#pragma omp parallel for schedule(static)
  for (int f = 0; f < m.F; ++f) v[f] = face(f);
  gather(m, s.data(), [&](double a, int f) { return a + v[f]; }, [&](double a, int f) { return a - v[f]; });
  for_slots(m, type, [&](int b, int t, int c) { s[c] += bnd(b, t, c); });
  return s;
}
// lduMatrix::negSumDiag
std::vector<double> neg_sum_diag(const M& m, const double* L, const double* U) {
  std::vector<double> s(m.C);
  gather(m, s.data(), [&](double a, int f) { return a - L[f]; }, [&](double a, int f) { return a - U[f]; });
  return s;
}

// ---------------------------------------------------------------- BC correction
// correct_boundary_conditions_scalar (dfMatrixOpBase.cu:2402-2450). Processor slots refresh
// only their [internal n] part here; the [neighbour n] part is the halo exchange's job.
void correct_bc_scalar(const M& m, const int* type, const double* vf, double* bvf, const Mix* mx = nullptr,
                       int comp = 0) {
  if (!mx)
    for (int b = 0; b < m.B; ++b)
      if (is_mixed(type[m.slot_patch[b]])) throw std::runtime_error("oracle: mixed boundary condition without its field data");
  const double* eg = has("boundary_heGradient") ? d("boundary_heGradient") : nullptr;
#pragma omp parallel for schedule(static)
  for (int b = 0; b < m.B; ++b) {
    int t = type[m.slot_patch[b]];
    int c = m.bfc[b];
    if (is_mixed(t)) {
      double f, ref;
      mix_vf_ref(t, *mx, b, m.B, comp, f, ref);
      bvf[b] = f * ref + (1.0 - f) * vf[c];
    } else if (t == ZG || t == EXTRAP) bvf[b] = vf[c];
    else if (t == CYCLIC) bvf[b] = interp_b(m.bw[b], vf[c], vf[m.partner_cell[b]]);
    else if (is_proc(t) && !m.primary[b]) bvf[b] = vf[c];
    else if (t == GRAD_E && eg)   // dfMatrixOpBase.cu:351-366
      bvf[b] = vf[c] + eg[b] / m.bdc[b];
  }
}
void correct_bc_vec(const M& m, const int* type, const double* vf, double* bvf, int ncomp, const Mix* mx = nullptr) {
  for (int k = 0; k < ncomp; ++k) correct_bc_scalar(m, type, vf + (long)k * m.C, bvf + (long)k * m.B, mx, k);
}

// face value of a scalar field on a boundary slot (linear interpolation semantics)
inline double bface(const M& m, int t, const double* vf, const double* bvf, int b, int c) {
  return is_coupled(t) ? interp_b(m.bw[b], vf[c], nbr(m, vf, bvf, b)) : bvf[b];
}

// ---------------------------------------------------------------- convection / interpolation schemes
// The reference GPU path hard-wires upwind for Yi and ha and linear for K and hDiffCorrFlux
// (dfYEqn.cu:543,587-593, dfEEqn.cu:166-174); its own cases ask for (system/fvSchemes of
// examples/dfLowMachFoam/notorch/threeD_reactingTGV/H2/cvodeIntegrator and
// test/dfLowMachFoam/twoD_reactingTGV/H2/cvodeSolver):
//   div(phi,Yi_h)       Gauss limitedLinear01 1   (the multivariate scheme YEqn.H:6-14 builds over the
//                                                  table createFields.H:118-129 = every Y_i plus he; EEqn.H
//                                                  reuses it for he)
//   div(phi,K)          Gauss limitedLinear 1     (fvc::div(phi, K), EEqn.H)
//   div(hDiffCorrFlux)  Gauss cubic               (fvc::div(hDiffCorrFlux), EEqn.H)
// Restated from OpenFOAM-7 (LimitedScheme::calcLimiter, Limited01.H / LimitedLimiter::limiter,
// limitedLinearLimiter, NVDTVD::r, multivariateScheme's min over the table's limiters,
// limitedSurfaceInterpolationScheme::weights, cubic::correction).
// "schemes" (int[3]): div(phi,Yi_h) 0 upwind | 2 limitedLinear | 3 limitedLinear01; div(phi,K) 0 upwind |
// 1 linear | 2 limitedLinear | 3 limitedLinear01; div(hDiffCorrFlux) 1 linear | 4 cubic. "scheme_k"
// (double[2]): the limiters' k for Yi_h and K. Absent: the GPU reference's schemes (0, 1, 1).
// div(phi,U) (int[3] of "schemes"): 1 linear (the GPU reference's) | 5 limitedLinearV (the 1D flame's,
// test/Tu500K-Phi1/system/fvSchemes: NVDVTVDV::r on grad(U), scheme_k[2])
enum Scheme { S_UPWIND = 0, S_LINEAR = 1, S_LL = 2, S_LL01 = 3, S_CUBIC = 4, S_LLV = 5 };
int scheme(int term) {
  static const int dflt[4] = {S_UPWIND, S_LINEAR, S_LINEAR, S_LINEAR};
  auto it = I.find("schemes");
  return it == I.end() ? dflt[term] : it->second[term];
}
double scheme_k(int term) { return has("scheme_k") ? d("scheme_k")[term] : 1.0; }
inline double pos0(double x) { return x >= 0 ? 1.0 : 0.0; }
inline double sgn(double x) { return x >= 0 ? 1.0 : -1.0; }   // OpenFOAM sign()

// limitedLinearLimiter<NVDTVD>::limiter, wrapped in Limited01Limiter (bounded01) when asked
double ll_limiter(double twoByk, bool bounded01, double faceFlux, double phiP, double phiN, const double* gP,
                  const double* gN, const double* dv) {
  if (bounded01 && ((faceFlux > 0 && (phiP < 0 || phiN > 1)) || (faceFlux < 0 && (phiN < 0 || phiP > 1)))) return 0;
  const double gradf = phiN - phiP;
  const double* g = faceFlux > 0 ? gP : gN;
  const double gradcf = dv[0] * g[0] + dv[1] * g[1] + dv[2] * g[2];
  double r;
  if (std::fabs(gradcf) >= 1000 * std::fabs(gradf)) r = 2 * 1000 * sgn(gradcf) * sgn(gradf) - 1;
  else r = 2 * (gradcf / gradf) - 1;
  return std::max(std::min(twoByk * r, 1.0), 0.0);
}

// per-field data the limiter reads at a face: values and Gauss-linear gradients [3][C] of the cells,
// and on coupled slots the neighbour-side value and gradient
struct LimField { const double *v, *bv, *g; const double* bg; };   // bg: neighbour-side gradient [3][B] (processor)

// weights of a limited scheme over `fields` (one field: LimitedScheme; several: multivariateScheme's min)
// -> w[F], bw[B]; every limiter evaluated in the same order, min over the table
void limited_weights(const M& m, const int* type, const std::vector<LimField>& fl, int kind, double k,
                     const double* phi, const double* bphi, double* w, double* bw) {
  const double twoByk = 2.0 / std::max(k, 1e-15);
  const bool b01 = kind == S_LL01;
  const double* md = d("mesh_distance");
  #pragma omp parallel for schedule(static)
  for (int f = 0; f < m.F; ++f) {
    const int o = m.own[f], n = m.nei[f];
    const double dv[3] = {md[f], md[(long)m.F + f], md[2L * m.F + f]};
    double lim = 1.0;
    for (size_t i = 0; i < fl.size(); ++i) {
      const LimField& x = fl[i];
      const double gP[3] = {x.g[o], x.g[(long)m.C + o], x.g[2L * m.C + o]};
      const double gN[3] = {x.g[n], x.g[(long)m.C + n], x.g[2L * m.C + n]};
      const double l = ll_limiter(twoByk, b01, phi[f], x.v[o], x.v[n], gP, gN, dv);
      lim = i == 0 ? l : std::min(lim, l);
    }
    w[f] = lim * m.w[f] + (1 - lim) * pos0(phi[f]);
  }
  const double* bd = d("boundary_delta");
  #pragma omp parallel for schedule(static)
  for (int b = 0; b < m.B; ++b) {
    const int t = type[m.slot_patch[b]];
    double lim = 1.0;
    if (is_coupled(t) && m.primary[b]) {
      const int c = m.bfc[b], pc = m.partner_cell[b];
      const double dv[3] = {bd[b], bd[(long)m.B + b], bd[2L * m.B + b]};
      for (size_t i = 0; i < fl.size(); ++i) {
        const LimField& x = fl[i];
        const double gP[3] = {x.g[c], x.g[(long)m.C + c], x.g[2L * m.C + c]};
        double gN[3];
        for (int q = 0; q < 3; ++q) gN[q] = pc >= 0 ? x.g[(long)q * m.C + pc] : x.bg[(long)q * m.B + b];
        const double l = ll_limiter(twoByk, b01, bphi[b], x.v[c], nbr(m, x.v, x.bv, b), gP, gN, dv);
        lim = i == 0 ? l : std::min(lim, l);
      }
    }
    bw[b] = lim * m.bw[b] + (1 - lim) * pos0(bphi[b]);
  }
}

void grad_scalar(const M& m, const int* type, const double* vf, const double* bvf, double* g, double* bg);

// limitedLinearV (limitedLinearLimiter<NVDVTVDV>): r from the velocity difference projected on
// d & grad(U) of the upwind cell; g the upwind cell's gradient tensor (row: direction, column: component)
double llv_limiter(double twoByk, double faceFlux, const double* vP, const double* vN, const double* g, const double* dv) {
  const double gv[3] = {vN[0] - vP[0], vN[1] - vP[1], vN[2] - vP[2]};
  const double gradf = gv[0] * gv[0] + gv[1] * gv[1] + gv[2] * gv[2];
  double dg[3];
  for (int j = 0; j < 3; ++j) dg[j] = dv[0] * g[j] + dv[1] * g[3 + j] + dv[2] * g[6 + j];
  const double gradcf = gv[0] * dg[0] + gv[1] * dg[1] + gv[2] * dg[2];
  double r;
  if (std::fabs(gradcf) >= 1000 * std::fabs(gradf)) r = 2 * 1000 * sgn(gradcf) * sgn(gradf) - 1;
  else r = 2 * (gradcf / gradf) - 1;
  (void)faceFlux;
  return std::max(std::min(twoByk * r, 1.0), 0.0);
}

// fvc::grad of a vector field (Gauss linear) -> g [9][C], g[i*3+j] = d U_j / d x_i
void grad_vector(const M& m, const int* tU, const double* U, const double* bU, double* g) {
  const long C = m.C, B = m.B;
  for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) {
    auto s = integrate(m, tU,
        [&](int f) { return m.sf(i, f) * interp_f(m.w[f], U[(long)j * C + m.own[f]], U[(long)j * C + m.nei[f]]); },
        [&](int b, int t, int c) { return m.bsf(i, b) * bface(m, t, U + (long)j * C, bU + (long)j * B, b, c); });
    #pragma omp parallel for schedule(static)
    for (int c = 0; c < C; ++c) g[(long)(i * 3 + j) * C + c] = s[c] / m.V[c];
  }
}

// weights of div(phi,U) with limitedLinearV from the cell gradients g [9][C] of U (fvc::grad(U))
void u_weights(const M& m, const int* tU, const double* U, const double* g, const double* phi, const double* bphi,
               double* w, double* bw) {
  const double twoByk = 2.0 / std::max(scheme_k(2), 1e-15);
  const double* md = d("mesh_distance");
  const long C = m.C;
  #pragma omp parallel for schedule(static)
  for (int f = 0; f < m.F; ++f) {
    const int o = m.own[f], n = m.nei[f];
    const double dv[3] = {md[f], md[(long)m.F + f], md[2L * m.F + f]};
    const double vP[3] = {U[o], U[C + o], U[2 * C + o]}, vN[3] = {U[n], U[C + n], U[2 * C + n]};
    const int cu = phi[f] > 0 ? o : n;
    double gu[9];
    for (int q = 0; q < 9; ++q) gu[q] = g[q * C + cu];
    const double lim = llv_limiter(twoByk, phi[f], vP, vN, gu, dv);
    w[f] = lim * m.w[f] + (1 - lim) * pos0(phi[f]);
  }
  const double* bd = d("boundary_delta");
  for (int b = 0; b < m.B; ++b) {
    const int t = tU[m.slot_patch[b]];
    double lim = 1.0;
    if (is_coupled(t) && m.primary[b]) {
      const int c = m.bfc[b], pc = m.partner_cell[b];
      if (pc < 0) throw std::runtime_error("oracle: limitedLinearV on processor patches is not supported");
      const double dv[3] = {bd[b], bd[(long)m.B + b], bd[2L * m.B + b]};
      const double vP[3] = {U[c], U[C + c], U[2 * C + c]}, vN[3] = {U[pc], U[C + pc], U[2 * C + pc]};
      const int cu = bphi[b] > 0 ? c : pc;
      double gu[9];
      for (int q = 0; q < 9; ++q) gu[q] = g[q * C + cu];
      lim = llv_limiter(twoByk, bphi[b], vP, vN, gu, dv);
    }
    bw[b] = lim * m.bw[b] + (1 - lim) * pos0(bphi[b]);
  }
}

// convection weights of div(phi,Yi_h): upwind (pos0(phi)), or the multivariate limited scheme over
// every Y_i and he (YEqn.H:6-14) -> "conv_w" [F], "boundary_conv_w" [B]; computed once per step at the
// start of YEqn and reused by EEqn (the same mvConvection object)
void conv_weights(const M& m) {
  const int* tY = ia("ptype_Y");
  const int* the = ia("ptype_he");
  double *phi = d("phi"), *bphi = d("boundary_phi"), *w = d("conv_w"), *bw = d("boundary_conv_w");
  const int kind = scheme(0);
  if (kind == S_UPWIND) {
    for (int f = 0; f < m.F; ++f) w[f] = pos0(phi[f]);
    for (int b = 0; b < m.B; ++b) bw[b] = pos0(bphi[b]);
    return;
  }
  if (kind != S_LL && kind != S_LL01) throw std::runtime_error("oracle: div(phi,Yi_h) scheme must be upwind or limitedLinear(01)");
  for (int b = 0; b < m.B; ++b)
    if (is_proc(tY[m.slot_patch[b]]) && !has("boundary_conv_grad"))
      throw std::runtime_error("oracle: limited div(phi,Yi_h) on processor patches needs boundary_conv_grad");
  const double *Y = d("Y"), *bY = d("boundary_Y"), *he = d("he"), *bhe = d("boundary_he");
  const double* bgx = has("boundary_conv_grad") ? d("boundary_conv_grad") : nullptr;   // [S+1][3][B]
  std::vector<double> g(3L * (m.S + 1) * m.C);
  std::vector<LimField> fl;
  for (int s = 0; s <= m.S; ++s) {
    const double* v = s < m.S ? Y + (long)s * m.C : he;
    const double* bv = s < m.S ? bY + (long)s * m.B : bhe;
    double* gs = g.data() + 3L * s * m.C;
    grad_scalar(m, s < m.S ? tY : the, v, bv, gs, nullptr);
    fl.push_back({v, bv, gs, bgx ? bgx + 3L * s * m.B : nullptr});
  }
  limited_weights(m, tY, fl, kind, scheme_k(0), phi, bphi, w, bw);
}

// interpolation weights of fvc::div(phi, K): linear (the mesh weights), upwind, or limitedLinear(01)
// from K's own Gauss gradient -> "K_w" [F], "boundary_K_w" [B]
void k_weights(const M& m, double* w, double* bw) {
  const int* tK = ia("ptype_K");
  double *phi = d("phi"), *bphi = d("boundary_phi");
  const int kind = scheme(1);
  if (kind == S_LINEAR) { std::copy(m.w, m.w + m.F, w); std::copy(m.bw, m.bw + m.B, bw); return; }
  if (kind == S_UPWIND) {
    for (int f = 0; f < m.F; ++f) w[f] = pos0(phi[f]);
    for (int b = 0; b < m.B; ++b) bw[b] = pos0(bphi[b]);
    return;
  }
  const double *K = d("K"), *bK = d("boundary_K");
  std::vector<double> g(3L * m.C);
  grad_scalar(m, tK, K, bK, g.data(), nullptr);
  const double* bg = has("boundary_gradK") ? d("boundary_gradK") : nullptr;
  limited_weights(m, tK, {LimField{K, bK, g.data(), bg}}, kind, scheme_k(1), phi, bphi, w, bw);
}

// cubic::correction of a vector field vf [3][C] (boundary bvf [3][B]) dotted with Sf: the face flux
// the scheme adds to the linear one (surfaceInterpolationScheme::dotInterpolate: + Sf & correction) ->
// cf [F], bcf [B] (0 on non-coupled slots, whose correction cubic zeroes)
void cubic_flux(const M& m, const int* type, const double* vf, const double* bvf, double* cf, double* bcf) {
  std::vector<double> g(9L * m.C);   // [3 comp][3 dir][C]: fvc::grad(vf.component(c))
  for (int c = 0; c < 3; ++c) grad_scalar(m, type, vf + (long)c * m.C, bvf + (long)c * m.B, g.data() + 3L * c * m.C, nullptr);
  const double* bgn = has("boundary_gradHD") ? d("boundary_gradHD") : nullptr;   // processor neighbour gradients [9][B]
  auto corr = [&](double lam, const double* S, double ms, double dc, const double* vP, const double* vN,
                  const double* gP, const double* gN) {
    const double kSc = lam * (1 - lam * (3 - 2 * lam));
    const double kVecP = ((1 - lam) * (1 - lam)) * lam;
    const double kVecN = (lam * lam) * (lam - 1);
    double cr[3];
    for (int c = 0; c < 3; ++c) {
      double v = kSc * vP[c] + (-kSc) * vN[c];
      double gi[3];
      for (int q = 0; q < 3; ++q) gi[q] = kVecP * gP[3 * c + q] + kVecN * gN[3 * c + q];
      cr[c] = v + (((gi[0] * S[0] + gi[1] * S[1] + gi[2] * S[2]) / ms) / dc);
    }
    return S[0] * cr[0] + S[1] * cr[1] + S[2] * cr[2];
  };
  #pragma omp parallel for schedule(static)
  for (int f = 0; f < m.F; ++f) {
    const int o = m.own[f], n = m.nei[f];
    const double S[3] = {m.sf(0, f), m.sf(1, f), m.sf(2, f)};
    double vP[3], vN[3], gP[9], gN[9];
    for (int c = 0; c < 3; ++c) { vP[c] = vf[(long)c * m.C + o]; vN[c] = vf[(long)c * m.C + n]; }
    for (int q = 0; q < 9; ++q) { gP[q] = g[(long)q * m.C + o]; gN[q] = g[(long)q * m.C + n]; }
    cf[f] = corr(m.w[f], S, m.magSf[f], m.dc[f], vP, vN, gP, gN);
  }
  #pragma omp parallel for schedule(static)
  for (int b = 0; b < m.B; ++b) {
    bcf[b] = 0.0;
    const int t = type[m.slot_patch[b]];
    if (!is_coupled(t) || !m.primary[b]) continue;
    const int c0 = m.bfc[b], pc = m.partner_cell[b];
    const double S[3] = {m.bsf(0, b), m.bsf(1, b), m.bsf(2, b)};
    double vP[3], vN[3], gP[9], gN[9];
    for (int c = 0; c < 3; ++c) { vP[c] = vf[(long)c * m.C + c0]; vN[c] = nbr(m, vf + (long)c * m.C, bvf + (long)c * m.B, b); }
    for (int q = 0; q < 9; ++q) {
      gP[q] = g[(long)q * m.C + c0];
      gN[q] = pc >= 0 ? g[(long)q * m.C + pc] : bgn[(long)q * m.B + b];
    }
    bcf[b] = corr(m.bw[b], S, m.bmagSf[b], m.bdc[b], vP, vN, gP, gN);
  }
}

// ---------------------------------------------------------------- rhoEqn (rhoEqn.H:33-45; dfRhoEqn.cu:41-92)
void rho_eqn(const M& m) {
  const int* trho = ia("ptype_rho");
  double *rho = d("rho"), *rho_old = d("rho_old"), *phi = d("phi"), *bphi = d("boundary_phi"), *brho = d("boundary_rho");
  auto div = integrate(m, trho, [&](int f) { return phi[f]; }, [&](int b, int, int) { return bphi[b]; });
  #pragma omp parallel for schedule(static)
  for (int c = 0; c < m.C; ++c) {
    double diag = m.rdt * m.V[c];                            // EulerDdtScheme::fvmDdt(vf)
    double src = m.rdt * rho_old[c] * m.V[c];
    src = src - div[c];                                      // + fvc::div(phi)
    rho[c] = src / diag;                                     // diagonal solver
    if (has("out_rho_diag")) { d("out_rho_diag")[c] = diag; d("out_rho_source")[c] = src; }
  }
  correct_bc_scalar(m, trho, rho, brho);
}

// ---------------------------------------------------------------- gradients (gaussGrad)
// fvc_grad_cell_scalar (dfMatrixOpBase.cu:1109-1195, 3004-3039) /V, then correctBC (:3085-3141)
void grad_scalar(const M& m, const int* type, const double* vf, const double* bvf, double* g, double* bg) {
  for (int k = 0; k < 3; ++k) {
    auto s = integrate(m, type, [&](int f) { return m.sf(k, f) * interp_f(m.w[f], vf[m.own[f]], vf[m.nei[f]]); },
                       [&](int b, int t, int c) { return m.bsf(k, b) * bface(m, t, vf, bvf, b, c); });
    #pragma omp parallel for schedule(static)
    for (int c = 0; c < m.C; ++c) g[(long)k * m.C + c] = s[c] / m.V[c];
  }
  if (!bg) return;
  #pragma omp parallel for schedule(static)
  for (int b = 0; b < m.B; ++b) {
    int t = type[m.slot_patch[b]];
    if (t == EMPTY) continue;
    int c = m.bfc[b];
    if (is_coupled(t)) {
      if (m.partner_cell[b] >= 0)
        for (int k = 0; k < 3; ++k) bg[(long)k * m.B + b] = interp_b(m.bw[b], g[(long)k * m.C + c], g[(long)k * m.C + m.partner_cell[b]]);
      else if (!m.primary[b]) for (int k = 0; k < 3; ++k) bg[(long)k * m.B + b] = g[(long)k * m.C + c];
      continue;
    }
    double nx = m.bsf(0, b) / m.bmagSf[b], ny = m.bsf(1, b) / m.bmagSf[b], nz = m.bsf(2, b) / m.bmagSf[b];
    double gx = g[c], gy = g[(long)m.C + c], gz = g[2L * m.C + c];
    double sn = (t == FV || t == CALC || t == FIX_E || is_mixed(t)) ? m.bdc[b] * (bvf[b] - vf[c]) : 0.0;
    double corr = sn - (nx * gx + ny * gy + nz * gz);
    bg[b] = gx + nx * corr; bg[(long)m.B + b] = gy + ny * corr; bg[2L * m.B + b] = gz + nz * corr;
  }
}

// ---------------------------------------------------------------- UEqn (UEqn.H:3-20; dfUEqn.cu:487-689)
// outputs: lower/upper/diag, source[3C] (UEqn.source()), source_solve[3C] (UEqn == -grad p),
// internal/boundary coeffs [3B], rAU, boundary_rAU
void u_eqn_assemble(const M& m) {
  const int* tU = ia("ptype_U");
  const int* tp = ia("ptype_p");
  const int* textr = ia("ptype_extrapolated");
  const int C = m.C, F = m.F, B = m.B;
  double *rho = d("rho"), *rho_old = d("rho_old"), *U_old = d("U_old"), *U = d("U"), *bU = d("boundary_U");
  double *phi = d("phi"), *bphi = d("boundary_phi"), *mu = d("mu"), *bmu = d("boundary_mu");
  double *p = d("p"), *bp = d("boundary_p");
  double *lower = d("out_lower"), *upper = d("out_upper"), *diag = d("out_diag"), *src = d("out_source");
  double *srcs = d("out_source_solve"), *ic = d("out_internal_coeffs"), *bc = d("out_boundary_coeffs");
  double *rAU = d("rAU"), *brAU = d("boundary_rAU");
  // fvc::grad(U) (fvc_grad_vector :944-1107): the explicit dev2 term's gradient, and limitedLinearV's
  std::vector<double> g(9L * C), bg(9L * B, 0.0), T(9L * C), bT(9L * B, 0.0);
  grad_vector(m, tU, U, bU, g.data());
  // fvm::div(phi,U) (gaussConvectionScheme::fvmDiv; dfMatrixOpBase.cu:741-781): Gauss linear, or the
  // limitedLinearV weights
  std::vector<double> wU(m.w, m.w + F), bwU(m.bw, m.bw + B);
  if (scheme(3) == S_LLV) u_weights(m, tU, U, g.data(), phi, bphi, wU.data(), bwU.data());
  std::vector<double> L1(F), U1(F), UL(F);
  #pragma omp parallel for schedule(static)
  for (int f = 0; f < F; ++f) { L1[f] = -wU[f] * phi[f]; U1[f] = L1[f] + phi[f]; }
  auto d1 = neg_sum_diag(m, L1.data(), U1.data());
  // fvm::laplacian(mu,U) (gaussLaplacianScheme; :783-810); symmetric
  #pragma omp parallel for schedule(static)
  for (int f = 0; f < F; ++f) UL[f] = m.dc[f] * (interp_f(m.w[f], mu[m.own[f]], mu[m.nei[f]]) * m.magSf[f]);
  auto dL = neg_sum_diag(m, UL.data(), UL.data());
  #pragma omp parallel for schedule(static)
  for (int f = 0; f < F; ++f) { lower[f] = L1[f] + (-UL[f]); upper[f] = U1[f] + (-UL[f]); }
  #pragma omp parallel for schedule(static)
  for (int c = 0; c < C; ++c) diag[c] = (m.rdt * rho[c] * m.V[c] + d1[c]) + (-dL[c]);
  std::fill(ic, ic + 3L * B, 0.0); std::fill(bc, bc + 3L * B, 0.0);
  const Mix mxU = mix_for("U");
  for_slots(m, tU, [&](int b, int t, int c) {
    double gam = is_coupled(t) ? interp_b(m.bw[b], mu[c], nbr(m, mu, bmu, b)) : bmu[b];
    double pG = gam * m.bmagSf[b];
    for (int k = 0; k < 3; ++k) {
      BCoef qc = bcoef_f(t, bU[(long)k * B + b], bwU[b], m.bdc[b], mxU, b, B, k);   // convection weights
      BCoef q = bcoef_f(t, bU[(long)k * B + b], m.bw[b], m.bdc[b], mxU, b, B, k);
      ic[(long)k * B + b] = bphi[b] * qc.vic + (-(pG * q.gic));
      bc[(long)k * B + b] = -bphi[b] * qc.vbc + (-(-pG * q.gbc));
    }
  });
  // -fvc::div(mu*dev2(T(fvc::grad(U)))) (scale_dev2T :623, fvc_div_cell_tensor :1625) on the gradient above
  #pragma omp parallel for schedule(static)
  for (int b = 0; b < B; ++b) {                           // boundary gradient, non-coupled only (:1239-1327)
    int t = tU[m.slot_patch[b]];
    if (t == EMPTY || is_coupled(t)) continue;
    int c = m.bfc[b];
    double nv[3] = {m.bsf(0, b) / m.bmagSf[b], m.bsf(1, b) / m.bmagSf[b], m.bsf(2, b) / m.bmagSf[b]};
    for (int j = 0; j < 3; ++j) {
      double sn = (t == FV || is_mixed(t)) ? m.bdc[b] * (bU[(long)j * B + b] - U[(long)j * C + c]) : 0.0;
      double gc[3] = {g[(long)(0 * 3 + j) * C + c], g[(long)(1 * 3 + j) * C + c], g[(long)(2 * 3 + j) * C + c]};
      double corr = sn - (nv[0] * gc[0] + nv[1] * gc[1] + nv[2] * gc[2]);
      for (int i = 0; i < 3; ++i) bg[(long)(i * 3 + j) * B + b] = gc[i] + nv[i] * corr;
    }
  }
  auto dev2T = [](double sc, const double* v, double* o) {   // mu*dev2(T(g)), scale_dev2t_tensor_kernel
    double tr = (2. / 3.) * (v[0] + v[4] + v[8]);
    o[0] = sc * (v[0] - tr); o[1] = sc * v[3]; o[2] = sc * v[6];
    o[3] = sc * v[1]; o[4] = sc * (v[4] - tr); o[5] = sc * v[7];
    o[6] = sc * v[2]; o[7] = sc * v[5]; o[8] = sc * (v[8] - tr);
  };
  #pragma omp parallel for schedule(static)
  for (int c = 0; c < C; ++c) {
    double v[9], o[9];
    for (int k = 0; k < 9; ++k) v[k] = g[(long)k * C + c];
    dev2T(mu[c], v, o);
    for (int k = 0; k < 9; ++k) T[(long)k * C + c] = o[k];
  }
  #pragma omp parallel for schedule(static)
  for (int b = 0; b < B; ++b) {
    double v[9], o[9];
    for (int k = 0; k < 9; ++k) v[k] = bg[(long)k * B + b];
    dev2T(bmu[b], v, o);
    for (int k = 0; k < 9; ++k) bT[(long)k * B + b] = o[k];
  }
  std::vector<double> divT[3];
  for (int j = 0; j < 3; ++j) {
    auto tf = [&](int i, int o, int n, double w) { return interp_f(w, T[(long)(i * 3 + j) * C + o], T[(long)(i * 3 + j) * C + n]); };
    divT[j] = integrate(m, tU,
        [&](int f) { int o = m.own[f], n = m.nei[f]; double w = m.w[f];
                     return m.sf(0, f) * tf(0, o, n, w) + m.sf(1, f) * tf(1, o, n, w) + m.sf(2, f) * tf(2, o, n, w); },
        [&](int b, int t, int c) {
          double tt[3];
          for (int i = 0; i < 3; ++i) {
            const double* Ti = T.data() + (long)(i * 3 + j) * C;
            tt[i] = is_coupled(t) ? interp_b(m.bw[b], Ti[c], nbr(m, Ti, bT.data() + (long)(i * 3 + j) * B, b))
                                  : bT[(long)(i * 3 + j) * B + b];
          }
          return m.bsf(0, b) * tt[0] + m.bsf(1, b) * tt[1] + m.bsf(2, b) * tt[2]; });
  }
  if (has("out_gradU")) std::copy(g.begin(), g.end(), d("out_gradU"));
  // source: ddt + divDevRhoReff explicit part
  for (int k = 0; k < 3; ++k)
    #pragma omp parallel for schedule(static)
    for (int c = 0; c < C; ++c) src[(long)k * C + c] = m.rdt * rho_old[c] * U_old[(long)k * C + c] * m.V[c] + divT[k][c];
  // UEqn == -fvc::grad(p)
  for (int k = 0; k < 3; ++k) {
    auto gp = integrate(m, tp, [&](int f) { return m.sf(k, f) * interp_f(m.w[f], p[m.own[f]], p[m.nei[f]]); },
                        [&](int b, int t, int c) { return m.bsf(k, b) * bface(m, t, p, bp, b, c); });
    #pragma omp parallel for schedule(static)
    for (int c = 0; c < C; ++c) srcs[(long)k * C + c] = src[(long)k * C + c] - gp[c];
  }
  // rAU = 1/UEqn.A() (fvMatrix::D + addCmptAvBoundaryDiag; dfUEqn.cu:721-738)
  #pragma omp parallel for schedule(static)
  for (int c = 0; c < C; ++c) rAU[c] = diag[c];
  for_slots(m, tU, [&](int b, int, int c) { rAU[c] += (ic[b] + ic[(long)B + b] + ic[2L * B + b]) / 3; });
  #pragma omp parallel for schedule(static)
  for (int c = 0; c < C; ++c) rAU[c] = 1 / (rAU[c] / m.V[c]);
  correct_bc_scalar(m, textr, rAU, brAU);
}

// HbyA = constrainHbyA(rAU*UEqn.H(), U, p) (fvMatrix::H; dfUEqn.cu:753-834)
void u_hbya(const M& m) {
  const int* tU = ia("ptype_U");
  const int* textr = ia("ptype_extrapolated");
  const int C = m.C, F = m.F, B = m.B;
  double *U = d("U"), *bU = d("boundary_U"), *rAU = d("rAU"), *brAU = d("boundary_rAU");
  double *lower = d("ueqn_lower"), *upper = d("ueqn_upper"), *src = d("ueqn_source");
  double *ic = d("ueqn_internal_coeffs"), *bc = d("ueqn_boundary_coeffs");
  double *H = d("HbyA"), *bH = d("boundary_HbyA");
  for (int k = 0; k < 3; ++k) {
    const double* Uk = U + (long)k * C;
    std::vector<double> bd(C, 0.0), Hl(C, 0.0);
    for_slots(m, tU, [&](int b, int, int c) { bd[c] += ic[(long)k * B + b]; });
    #pragma omp parallel for schedule(static)
    for (int c = 0; c < C; ++c) bd[c] = -bd[c];
    for_slots(m, tU, [&](int b, int, int c) { bd[c] += (ic[b] + ic[(long)B + b] + ic[2L * B + b]) / 3; });
    gather(m, Hl.data(), [&](double a, int f) { return a - upper[f] * Uk[m.nei[f]]; },   // lduMatrix::H
           [&](double a, int f) { return a - lower[f] * Uk[m.own[f]]; });
    double* Hk = H + (long)k * C;
    #pragma omp parallel for schedule(static)
    for (int c = 0; c < C; ++c) Hk[c] = bd[c] * Uk[c] + (Hl[c] + src[(long)k * C + c]);
    for_slots(m, tU, [&](int b, int t, int c) {         // addBoundarySource
      Hk[c] += is_coupled(t) ? bc[(long)k * B + b] * nbr(m, Uk, bU + (long)k * B, b) : bc[(long)k * B + b];
    });
    #pragma omp parallel for schedule(static)
    for (int c = 0; c < C; ++c) Hk[c] = Hk[c] / m.V[c];
  }
  correct_bc_vec(m, textr, H, bH, 3);
  for (int k = 0; k < 3; ++k) {
    #pragma omp parallel for schedule(static)
    for (int c = 0; c < C; ++c) H[(long)k * C + c] = rAU[c] * H[(long)k * C + c];
    #pragma omp parallel for schedule(static)
    for (int b = 0; b < B; ++b) {
      int t = tU[m.slot_patch[b]];
      bH[(long)k * B + b] = brAU[b] * bH[(long)k * B + b];
      if (t == FV) bH[(long)k * B + b] = bU[(long)k * B + b];   // constrainHbyA
    }
  }
}

// ---------------------------------------------------------------- pEqn (pEqn.H:1-129; dfpEqn.cu:379-546)
void p_eqn_assemble(const M& m) {
  const int* tU = ia("ptype_U");
  const int* tp = ia("ptype_p");
  const int C = m.C, F = m.F, B = m.B;
  double *rho = d("rho"), *brho = d("boundary_rho"), *rho_old = d("rho_old"), *brho_old = d("boundary_rho_old");
  double *rAU = d("rAU"), *brAU = d("boundary_rAU"), *H = d("HbyA"), *bH = d("boundary_HbyA");
  double *U_old = d("U_old"), *bU_old = d("boundary_U_old"), *phi_old = d("phi_old"), *bphi_old = d("boundary_phi_old");
  double *p = d("p"), *bp = d("boundary_p"), *p_old = d("p_old"), *psi = d("psi");
  double *lower = d("out_lower"), *upper = d("out_upper"), *diag = d("out_diag"), *src = d("out_source");
  double *ic = d("out_internal_coeffs"), *bc = d("out_boundary_coeffs");
  double *rf = d("out_rhorAUf"), *brf = d("out_boundary_rhorAUf");
  double *ph = d("out_phiHbyA"), *bph = d("out_boundary_phiHbyA");
  const double small_ = 1e-15;    // OpenFOAM 'small' in ddtScheme::fvcDdtPhiCoeff
  const double* dscale = has("study_ddtcorr_scale") ? d("study_ddtcorr_scale") : nullptr;
  // rhorAUf = fvc::interpolate(rho*rAU)
  std::vector<double> rr(C), rUo(3L * C);
  #pragma omp parallel for schedule(static)
  for (int c = 0; c < C; ++c) rr[c] = rho[c] * rAU[c];
  for (int k = 0; k < 3; ++k) for (int c = 0; c < C; ++c) rUo[(long)k * C + c] = rho_old[c] * U_old[(long)k * C + c];
  #pragma omp parallel for schedule(static)
  for (int f = 0; f < F; ++f) rf[f] = interp_f(m.w[f], rr[m.own[f]], rr[m.nei[f]]);
  std::fill(brf, brf + B, 0.0); std::fill(bph, bph + B, 0.0);
  for_slots(m, tp, [&](int b, int t, int c) {
    brf[b] = is_coupled(t) ? interp_b(m.bw[b], rr[c], m.partner_cell[b] >= 0 ? rr[m.partner_cell[b]] : brho[b] * brAU[b])
                           : brho[b] * brAU[b];
  });
  // phiHbyA = interpolate(rho)*flux(HbyA) + rhorAUf*ddtCorr(rho, U, phi) (EulerDdtScheme::fvcDdtPhiCorr)
  #pragma omp parallel for schedule(static)
  for (int f = 0; f < F; ++f) {
    int o = m.own[f], n = m.nei[f];
    double w = m.w[f];
    double phiCorr = phi_old[f] - (m.sf(0, f) * interp_f(w, rUo[o], rUo[n]) + m.sf(1, f) * interp_f(w, rUo[C + o], rUo[C + n]) +
                                   m.sf(2, f) * interp_f(w, rUo[2L * C + o], rUo[2L * C + n]));
    double coeff = 1.0 - std::min(std::fabs(phiCorr) / (std::fabs(phi_old[f]) + small_), 1.0);
    double ddtCorr = coeff * m.rdt * phiCorr;
    if (dscale) ddtCorr = ddtCorr * *dscale;   // sensitivity study only (CPU-A DFMI_CPUA_STUDY ddtcorr=)
    double fl = m.sf(0, f) * interp_f(w, H[o], H[n]) + m.sf(1, f) * interp_f(w, H[C + o], H[C + n]) +
                m.sf(2, f) * interp_f(w, H[2L * C + o], H[2L * C + n]);
    ph[f] = interp_f(w, rho[o], rho[n]) * fl + rf[f] * ddtCorr;
  }
  for_slots(m, tp, [&](int b, int t, int c) {
    int tu = tU[m.slot_patch[b]];
    double ruo[3], Hb[3], rb;
    for (int k = 0; k < 3; ++k) {
      if (is_coupled(tu)) {
        double rn = m.partner_cell[b] >= 0 ? rUo[(long)k * C + m.partner_cell[b]] : brho_old[b] * bU_old[(long)k * B + b];
        ruo[k] = interp_b(m.bw[b], rUo[(long)k * C + c], rn);
        Hb[k] = interp_b(m.bw[b], H[(long)k * C + c], nbr(m, H + (long)k * C, bH + (long)k * B, b));
      } else { ruo[k] = brho_old[b] * bU_old[(long)k * B + b]; Hb[k] = bH[(long)k * B + b]; }
    }
    rb = is_coupled(tu) ? interp_b(m.bw[b], rho[c], nbr(m, rho, brho, b)) : brho[b];
    double phiCorr = bphi_old[b] - (m.bsf(0, b) * ruo[0] + m.bsf(1, b) * ruo[1] + m.bsf(2, b) * ruo[2]);
    double coeff = fixes_value(tu) ? 0.0 : 1.0 - std::min(std::fabs(phiCorr) / (std::fabs(bphi_old[b]) + small_), 1.0);
    double fl = m.bsf(0, b) * Hb[0] + m.bsf(1, b) * Hb[1] + m.bsf(2, b) * Hb[2];
    bph[b] = rb * fl + brf[b] * (dscale ? (coeff * m.rdt * phiCorr) * *dscale : coeff * m.rdt * phiCorr);
  });
  // fvm::laplacian(rhorAUf, p), symmetric
  std::vector<double> UL(F);
  #pragma omp parallel for schedule(static)
  for (int f = 0; f < F; ++f) UL[f] = m.dc[f] * (rf[f] * m.magSf[f]);
  auto dL = neg_sum_diag(m, UL.data(), UL.data());
  auto div = integrate(m, tp, [&](int f) { return ph[f]; }, [&](int b, int, int) { return bph[b]; });
  #pragma omp parallel for schedule(static)
  for (int c = 0; c < C; ++c) {
    // psi*correction(fvm::ddt(p)) (correct_diag_mtx_multi_tpsi_kernel, dfpEqn.cu:258)
    double dg = m.rdt * m.V[c];
    double sr = m.rdt * p_old[c] * m.V[c];
    double APsi = -dg * p[c] + sr;
    sr = sr - APsi;
    sr = sr * psi[c]; dg = dg * psi[c];
    // fvc::ddt(rho) + ... + fvc::div(phiHbyA)
    sr = sr - m.V[c] * (m.rdt * (rho[c] - rho_old[c]));
    sr = sr - div[c];
    src[c] = sr;
    diag[c] = dg - dL[c];                                   // - fvm::laplacian
  }
  #pragma omp parallel for schedule(static)
  for (int f = 0; f < F; ++f) { lower[f] = -UL[f]; upper[f] = -UL[f]; }
  std::fill(ic, ic + B, 0.0); std::fill(bc, bc + B, 0.0);
  const Mix mxP = mix_for("p");
  for_slots(m, tp, [&](int b, int t, int) {
    BCoef q;
    if (t == WAVE) {   // advectiveFvPatchField::updateCoeffs (Euler), waveTransmissive::advectionSpeed
      const double* bph_now = d("boundary_phi");
      double wsp = bph_now[b] / (brho[b] * m.bmagSf[b]) + std::sqrt(d("boundary_p_gamma")[b] / d("boundary_psi")[b]);
      wsp = std::fmax(wsp, 0.0);
      double vf = 1.0 / (1.0 + wsp * (1.0 / m.rdt) * m.bdc[b]);
      d("boundary_p_vf")[b] = vf;
      double ref = mxP.wref[b];
      q = {1.0 - vf, vf * ref, -vf * m.bdc[b], vf * m.bdc[b] * ref};
    } else q = bcoef_f(t, bp[b], m.bw[b], m.bdc[b], mxP, b, B, 0);
    double pG = brf[b] * m.bmagSf[b];
    ic[b] = -(pG * q.gic);
    bc[b] = -(-pG * q.gbc);
  });
}

// after the p solve: phi = phiHbyA + pEqn.flux(); U = HbyA - rAU*grad(p); K; dpdt (dfpEqn.cu:506-533)
void p_eqn_post(const M& m) {
  const int* tU = ia("ptype_U");
  const int* tp = ia("ptype_p");
  const int C = m.C, F = m.F, B = m.B;
  double *p = d("p"), *bp = d("boundary_p"), *p_old = d("p_old");
  double *lower = d("peqn_lower"), *upper = d("peqn_upper"), *ic = d("peqn_internal_coeffs"), *bc = d("peqn_boundary_coeffs");
  double *ph = d("peqn_phiHbyA"), *bph = d("peqn_boundary_phiHbyA");
  double *phi = d("phi"), *bphi = d("boundary_phi"), *U = d("U"), *bU = d("boundary_U");
  double *H = d("HbyA"), *rAU = d("rAU"), *K = d("K"), *bK = d("boundary_K"), *dpdt = d("dpdt");
  { const Mix mx = mix_for("p"); correct_bc_scalar(m, tp, p, bp, &mx); }
  #pragma omp parallel for schedule(static)
  for (int f = 0; f < F; ++f) phi[f] = ph[f] + (upper[f] * p[m.nei[f]] - lower[f] * p[m.own[f]]);  // lduMatrix::faceH
  for_slots(m, tp, [&](int b, int t, int c) {              // fvMatrix::flux boundary
    double fl = is_coupled(t) ? ic[b] * p[c] - bc[b] * nbr(m, p, bp, b) : ic[b] * p[c] - bc[b];
    bphi[b] = bph[b] + fl;
  });
  std::vector<double> g(3L * C);
  grad_scalar(m, tp, p, bp, g.data(), nullptr);
  for (int k = 0; k < 3; ++k)
    #pragma omp parallel for schedule(static)
    for (int c = 0; c < C; ++c) U[(long)k * C + c] = H[(long)k * C + c] - rAU[c] * g[(long)k * C + c];
  { const Mix mx = mix_for("U"); correct_bc_vec(m, tU, U, bU, 3, &mx); }
  #pragma omp parallel for schedule(static)
  for (int c = 0; c < C; ++c) K[c] = 0.5 * (U[c] * U[c] + U[(long)C + c] * U[(long)C + c] + U[2L * C + c] * U[2L * C + c]);
  #pragma omp parallel for schedule(static)
  for (int b = 0; b < B; ++b) bK[b] = 0.5 * (bU[b] * bU[b] + bU[(long)B + b] * bU[(long)B + b] + bU[2L * B + b] * bU[2L * B + b]);
  #pragma omp parallel for schedule(static)
  for (int c = 0; c < C; ++c) dpdt[c] = m.rdt * (p[c] - p_old[c]);
}

// ---------------------------------------------------------------- YEqn preparation (YEqn.H:24-118; dfYEqn.cu:443-552)
void y_prep(const M& m) {
  const int* tY = ia("ptype_Y");
  const int S = m.S, C = m.C, F = m.F, B = m.B;
  double *Y = d("Y"), *bY = d("boundary_Y"), *rhoD = d("rhoD"), *brhoD = d("boundary_rhoD"), *hai = d("hai"),
         *bhai = d("boundary_hai"), *alpha = d("alpha"), *balpha = d("boundary_alpha");
  double *dAD = d("diffAlphaD"), *hD = d("hDiffCorrFlux"), *bhD = d("boundary_hDiffCorrFlux");
  double *sumE = d("sumYDiffError"), *bsumE = d("boundary_sumYDiffError");
  std::vector<double> g(3L * S * C), bg(3L * S * B, 0.0);
  for (int s = 0; s < S; ++s) grad_scalar(m, tY, Y + (long)s * C, bY + (long)s * B, g.data() + 3L * s * C, bg.data() + 3L * s * B);
  if (has("out_gradY")) std::copy(g.begin(), g.end(), d("out_gradY"));
  // sumYDiffError = sum_i rhoD_i*grad(Y_i); boundary field = product of boundary fields
  auto fold_sum = [&](int n, const double* rd, const double* gy, double* se) {
    #pragma omp parallel for collapse(2) schedule(static)
    for (int k = 0; k < 3; ++k) for (int i = 0; i < n; ++i) {
      double a = 0.0;
      for (int s = 0; s < S; ++s) a += rd[(long)s * n + i] * gy[(long)n * s * 3 + (long)n * k + i];
      se[(long)k * n + i] = a;
    }
  };
  fold_sum(C, rhoD, g.data(), sumE);
  fold_sum(B, brhoD, bg.data(), bsumE);
  // hDiffCorrFlux = sum_i hai_i*(rhoD_i*grad(Y_i) - Y_i*sumYDiffError)
  auto fold_h = [&](int n, const double* ha, const double* rd, const double* y, const double* gy, const double* se, double* hd) {
    #pragma omp parallel for collapse(2) schedule(static)
    for (int k = 0; k < 3; ++k) for (int i = 0; i < n; ++i) {
      double a = 0.0;
      for (int s = 0; s < S; ++s) {
        long si = (long)s * n + i;
        a += ha[si] * (rd[si] * gy[(long)n * s * 3 + (long)n * k + i] - y[si] * se[(long)k * n + i]);
      }
      hd[(long)k * n + i] = a;
    }
  };
  fold_h(C, hai, rhoD, Y, g.data(), sumE, hD);
  fold_h(B, bhai, brhoD, bY, bg.data(), bsumE, bhD);
  // diffAlphaD = sum_i fvc::laplacian(alpha*hai_i, Y_i) (per species /V, then accumulated)
  std::fill(dAD, dAD + C, 0.0);
  std::vector<double> ah(C);
  for (int s = 0; s < S; ++s) {
    const double *y = Y + (long)s * C, *by = bY + (long)s * B, *hs = hai + (long)s * C, *bhs = bhai + (long)s * B;
    #pragma omp parallel for schedule(static)
    for (int c = 0; c < C; ++c) ah[c] = alpha[c] * hs[c];
    auto lap = integrate(m, tY,
        [&](int f) { int o = m.own[f], n = m.nei[f];
                     return interp_f(m.w[f], ah[o], ah[n]) * m.magSf[f] * (m.dc[f] * (y[n] - y[o])); },
        [&](int b, int t, int c) {
          if (is_coupled(t)) {
            double an = m.partner_cell[b] >= 0 ? ah[m.partner_cell[b]] : balpha[b] * bhs[b];
            return interp_b(m.bw[b], ah[c], an) * m.bmagSf[b] * (m.bdc[b] * (nbr(m, y, by, b) - y[c]));
          }
          double sng = (t == FV || t == CALC || t == FIX_E || is_mixed(t)) ? m.bdc[b] * (by[b] - y[c]) : 0.0;
          return balpha[b] * bhs[b] * m.bmagSf[b] * sng; });
    #pragma omp parallel for schedule(static)
    for (int c = 0; c < C; ++c) dAD[c] = dAD[c] + lap[c] / m.V[c];
  }
}

// ---------------------------------------------------------------- Y species matrices (YEqn.H:99-118)
// out_* are [S][*]; the inert species is left zero. phiUc = linearInterpolate(sumYDiffError) & Sf.
void y_assemble(const M& m) {
  const int* tY = ia("ptype_Y");
  const int inert = ia("inert_index")[0];
  const int S = m.S, C = m.C, F = m.F, B = m.B;
  double *Y = d("Y"), *bY = d("boundary_Y"), *rhoD = d("rhoD"), *brhoD = d("boundary_rhoD"), *RR = d("RR");
  double *rho = d("rho"), *rho_old = d("rho_old"), *phi = d("phi"), *bphi = d("boundary_phi");
  double *sumE = d("sumYDiffError"), *bsumE = d("boundary_sumYDiffError");
  double *lo = d("out_lower"), *up = d("out_upper"), *dg = d("out_diag"), *sr = d("out_source");
  double *icA = d("out_internal_coeffs"), *bcA = d("out_boundary_coeffs");
  std::vector<double> phiUc(F), bphiUc(B, 0.0);
  #pragma omp parallel for schedule(static)
  for (int f = 0; f < F; ++f) {
    int o = m.own[f], n = m.nei[f];
    double w = m.w[f];
    phiUc[f] = m.sf(0, f) * interp_f(w, sumE[o], sumE[n]) + m.sf(1, f) * interp_f(w, sumE[C + o], sumE[C + n]) +
               m.sf(2, f) * interp_f(w, sumE[2L * C + o], sumE[2L * C + n]);
  }
  for_slots(m, tY, [&](int b, int t, int c) {
    double e[3];
    for (int k = 0; k < 3; ++k)
      e[k] = is_coupled(t) ? interp_b(m.bw[b], sumE[(long)k * C + c], nbr(m, sumE + (long)k * C, bsumE + (long)k * B, b))
                           : bsumE[(long)k * B + b];
    bphiUc[b] = m.bsf(0, b) * e[0] + m.bsf(1, b) * e[1] + m.bsf(2, b) * e[2];
  });
  if (has("out_phiUc")) { std::copy(phiUc.begin(), phiUc.end(), d("out_phiUc")); std::copy(bphiUc.begin(), bphiUc.end(), d("out_boundary_phiUc")); }
  // multivariate Gauss convection: the same weights (upwind pos0(phi), or the limited scheme's from
  // conv_weights) for both fluxes -- multivariateGaussConvectionScheme::fvmDiv(phiUc, Yi) interpolates
  // with the weights the scheme computed from phi
  const double* cw = has("conv_w") ? d("conv_w") : nullptr;
  const double* bcw = has("conv_w") ? d("boundary_conv_w") : nullptr;
  std::vector<double> L1(F), U1(F), L2(F), U2(F), UL(F);
  #pragma omp parallel for schedule(static)
  for (int f = 0; f < F; ++f) {
    double w = cw ? cw[f] : (phi[f] >= 0 ? 1.0 : 0.0);
    L1[f] = -w * phi[f]; U1[f] = L1[f] + phi[f];
    L2[f] = -w * phiUc[f]; U2[f] = L2[f] + phiUc[f];
  }
  auto d1 = neg_sum_diag(m, L1.data(), U1.data());
  auto d2 = neg_sum_diag(m, L2.data(), U2.data());
  std::fill(lo, lo + (long)S * F, 0.0); std::fill(up, up + (long)S * F, 0.0);
  std::fill(dg, dg + (long)S * C, 0.0); std::fill(sr, sr + (long)S * C, 0.0);
  std::fill(icA, icA + (long)S * B, 0.0); std::fill(bcA, bcA + (long)S * B, 0.0);
  const Mix mxY = mix_for("Y");
  for (int s = 0; s < S; ++s) {
    if (s == inert) continue;
    const double *rd = rhoD + (long)s * C, *brd = brhoD + (long)s * B, *y = Y + (long)s * C, *by = bY + (long)s * B;
    #pragma omp parallel for schedule(static)
    for (int f = 0; f < F; ++f) UL[f] = m.dc[f] * (interp_f(m.w[f], rd[m.own[f]], rd[m.nei[f]]) * m.magSf[f]);
    auto dL = neg_sum_diag(m, UL.data(), UL.data());
    #pragma omp parallel for schedule(static)
    for (int f = 0; f < F; ++f) {
      lo[(long)s * F + f] = (L1[f] + L2[f]) - UL[f];
      up[(long)s * F + f] = (U1[f] + U2[f]) - UL[f];
    }
    #pragma omp parallel for schedule(static)
    for (int c = 0; c < C; ++c) {
      dg[(long)s * C + c] = (m.rdt * rho[c] * m.V[c] + (d1[c] + d2[c])) - dL[c];
      sr[(long)s * C + c] = m.rdt * rho_old[c] * y[c] * m.V[c] + m.V[c] * RR[(long)s * C + c];
    }
    for_slots(m, tY, [&](int b, int t, int c) {
      double wu = bcw ? bcw[b] : (bphi[b] >= 0 ? 1.0 : 0.0);
      BCoef qc = bcoef_f(t, by[b], wu, m.bdc[b], mxY, b, B, s);
      BCoef ql = bcoef_f(t, by[b], m.bw[b], m.bdc[b], mxY, b, B, s);
      double gam = is_coupled(t) ? interp_b(m.bw[b], rd[c], nbr(m, rd, brd, b)) : brd[b];
      double pG = gam * m.bmagSf[b];
      icA[(long)s * B + b] = (bphi[b] * qc.vic + bphiUc[b] * qc.vic) - pG * ql.gic;
      bcA[(long)s * B + b] = (-bphi[b] * qc.vbc + -bphiUc[b] * qc.vbc) - (-pG * ql.gbc);
    });
  }
}

// Y[inert] = max(1 - sum, 0) after clipping (yeqn_compute_y_inertIndex_kernel, dfYEqn.cu:281-298)
void y_inert(const M& m) {
  const int inert = ia("inert_index")[0];
  const int* tY = ia("ptype_Y");
  double *Y = d("Y"), *bY = d("boundary_Y");
  #pragma omp parallel for schedule(static)
  for (int c = 0; c < m.C; ++c) {
    double sum = 0;
    for (int s = 0; s < m.S; ++s) {
      if (s == inert) continue;
      double yi = Y[(long)s * m.C + c];
      yi = yi > 0 ? yi : 0;
      Y[(long)s * m.C + c] = yi;
      sum += yi;
    }
    sum = 1 - sum;
    Y[(long)inert * m.C + c] = sum > 0 ? sum : 0;
  }
  const Mix mx = mix_for("Y");
  for (int s = 0; s < m.S; ++s) correct_bc_scalar(m, tY, Y + (long)s * m.C, bY + (long)s * m.B, &mx, s);
}

// ---------------------------------------------------------------- EEqn (EEqn.H:12-45; dfEEqn.cu:108-264)
void e_assemble(const M& m) {
  const int* the = ia("ptype_he");
  const int* tK = ia("ptype_K");
  const int C = m.C, F = m.F, B = m.B;
  double *he = d("he"), *bhe = d("boundary_he"), *rho = d("rho"), *rho_old = d("rho_old"), *K = d("K"),
         *K_old = d("K_old"), *bK = d("boundary_K"), *phi = d("phi"), *bphi = d("boundary_phi"), *alpha = d("alpha"),
         *balpha = d("boundary_alpha"), *hD = d("hDiffCorrFlux"), *bhD = d("boundary_hDiffCorrFlux"),
         *dpdt = d("dpdt"), *dAD = d("diffAlphaD");
  double *lower = d("out_lower"), *upper = d("out_upper"), *diag = d("out_diag"), *src = d("out_source");
  double *ic = d("out_internal_coeffs"), *bc = d("out_boundary_coeffs");
  const double* egrad = has("boundary_heGradient") ? d("boundary_heGradient") : nullptr;
  // he convection: mvConvection->fvmDiv(phi, he) (EEqn.H), the weights YEqn's scheme computed
  const double* cw = has("conv_w") ? d("conv_w") : nullptr;
  const double* bcw = has("conv_w") ? d("boundary_conv_w") : nullptr;
  std::vector<double> L1(F), U1(F), UL(F);
  #pragma omp parallel for schedule(static)
  for (int f = 0; f < F; ++f) { double w = cw ? cw[f] : (phi[f] >= 0 ? 1.0 : 0.0); L1[f] = -w * phi[f]; U1[f] = L1[f] + phi[f]; }
  auto d1 = neg_sum_diag(m, L1.data(), U1.data());
  #pragma omp parallel for schedule(static)
  for (int f = 0; f < F; ++f) UL[f] = m.dc[f] * (interp_f(m.w[f], alpha[m.own[f]], alpha[m.nei[f]]) * m.magSf[f]);
  auto dL = neg_sum_diag(m, UL.data(), UL.data());
  // fvc::div(phi, K): interpolation weights of div(phi,K) (linear: the mesh weights)
  std::vector<double> kw(m.w, m.w + F), bkw(m.bw, m.bw + B);
  if (scheme(1) != S_LINEAR) k_weights(m, kw.data(), bkw.data());
  auto divK = integrate(m, tK, [&](int f) { return phi[f] * interp_f(kw[f], K[m.own[f]], K[m.nei[f]]); },
                        [&](int b, int t, int c) {
                          return bphi[b] * (is_coupled(t) ? interp_b(bkw[b], K[c], nbr(m, K, bK, b)) : bK[b]); });
  // fvc::div(hDiffCorrFlux): linear, plus cubic's explicit correction (Sf & correction)
  const bool cubic = scheme(2) == S_CUBIC;
  std::vector<double> cf, bcf;
  if (cubic) {
    cf.assign(F, 0.0); bcf.assign(B, 0.0);
    cubic_flux(m, ia("ptype_calculated"), hD, bhD, cf.data(), bcf.data());
  }
  auto divh = integrate(m, the,
      [&](int f) { int o = m.own[f], n = m.nei[f]; double w = m.w[f];
                   double v = m.sf(0, f) * interp_f(w, hD[o], hD[n]) + m.sf(1, f) * interp_f(w, hD[C + o], hD[C + n]) +
                              m.sf(2, f) * interp_f(w, hD[2L * C + o], hD[2L * C + n]);
                   return cubic ? v + cf[f] : v; },
      [&](int b, int t, int c) {
        double h[3];
        for (int k = 0; k < 3; ++k) h[k] = bface(m, t, hD + (long)k * C, bhD + (long)k * B, b, c);
        double v = m.bsf(0, b) * h[0] + m.bsf(1, b) * h[1] + m.bsf(2, b) * h[2];
        return (cubic && is_coupled(t)) ? v + bcf[b] : v; });
  #pragma omp parallel for schedule(static)
  for (int f = 0; f < F; ++f) { lower[f] = L1[f] - UL[f]; upper[f] = U1[f] - UL[f]; }
  #pragma omp parallel for schedule(static)
  for (int c = 0; c < C; ++c) {
    double V = m.V[c];
    diag[c] = (m.rdt * rho[c] * V + d1[c]) - dL[c];
    double sL = m.rdt * rho_old[c] * he[c] * V;
    sL = sL - V * (m.rdt * (rho[c] * K[c] - rho_old[c] * K_old[c]));   // + fvc::ddt(rho,K)
    sL = sL - divK[c];                                                // + fvc::div(phi,K)
    sL = sL + V * dpdt[c];                                            // - dpdt
    double sR = V * dAD[c];                                           // laplacian - diffAlphaD
    sR = sR - divh[c];                                                // + fvc::div(hDiffCorrFlux)
    src[c] = sL - sR;
  }
  std::fill(ic, ic + B, 0.0); std::fill(bc, bc + B, 0.0);
  for_slots(m, the, [&](int b, int t, int c) {
    double eg = egrad ? egrad[b] : 0.0;
    BCoef qc = bcoef(t, bhe[b], bcw ? bcw[b] : (bphi[b] >= 0 ? 1.0 : 0.0), m.bdc[b], eg);
    BCoef ql = bcoef(t, bhe[b], m.bw[b], m.bdc[b], eg);
    double gam = is_coupled(t) ? interp_b(m.bw[b], alpha[c], nbr(m, alpha, balpha, b)) : balpha[b];
    double pG = gam * m.bmagSf[b];
    ic[b] = bphi[b] * qc.vic - pG * ql.gic;
    bc[b] = -bphi[b] * qc.vbc - (-pG * ql.gbc);
  });
}

// ---------------------------------------------------------------- thermo (dfThermo.cu:54-357, 572-671)
struct Thermo { int S; std::vector<double> W, nasa, visc, cond, bdiff, vc1, vc2; };
Thermo g_th;
const double R_GAS = 8314.46261815324;
const double SQRT8 = 2.8284271247461903;

double h_mix(const Thermo& th, double T, const double* y, long ys) {    // calculate_enthalpy_device_kernel (:257)
  double h = 0.;
  for (int i = 0; i < th.S; ++i) {
    const double* a = &th.nasa[i * 15];
    int o = (T > a[0]) ? 1 : 8;
    h += (a[o] + a[o + 1] * T / 2 + a[o + 2] * T * T / 3 + a[o + 3] * T * T * T / 4 + a[o + 4] * T * T * T * T / 5 +
          a[o + 5] / T) * R_GAS * T / th.W[i] * y[i * ys];
  }
  return h;
}
double cp_mix(const Thermo& th, double T, const double* y, long ys) {   // calculate_cp_device_kernel (:153)
  double cp = 0.;
  for (int i = 0; i < th.S; ++i) {
    const double* a = &th.nasa[i * 15];
    int o = (T > a[0]) ? 1 : 8;
    cp += y[i * ys] * (a[o] + a[o + 1] * T + a[o + 2] * T * T + a[o + 3] * T * T * T + a[o + 4] * T * T * T * T) * R_GAS / th.W[i];
  }
  return cp;
}
double h_species(const Thermo& th, int i, double T) {     // hai_i = h0_i(T) per unit mass (dfChemistryModel.C:531-539)
  const double* a = &th.nasa[i * 15];
  int o = (T > a[0]) ? 1 : 8;
  return (a[o] + a[o + 1] * T / 2 + a[o + 2] * T * T / 3 + a[o + 3] * T * T * T / 4 + a[o + 4] * T * T * T * T / 5 +
          a[o + 5] / T) * R_GAS * T / th.W[i];
}

void thermo_point(const Thermo& th, bool fixT, double& T, double& he, double p, const double* y, long ys,
                  double& psi, double& rho, double& mu, double& alpha, double* rhoD, double* hai, long os) {
  const int S = th.S;
  double X[64];
  double sum = 0.;
  for (int i = 0; i < S; ++i) sum += y[i * ys] / th.W[i];
  double Wm = 0.;
  for (int i = 0; i < S; ++i) { X[i] = y[i * ys] / (th.W[i] * sum); Wm += X[i] * th.W[i]; }
  if (fixT) he = h_mix(th, T, y, ys);
  else {                                                   // Newton, atol = rtol = 1e-7, <= 20 its (:296-323)
    double t = T;
    for (int n = 0; n < 20; ++n) {
      double h = h_mix(th, t, y, ys), cp = cp_mix(th, t, y, ys);
      double dT = (h - he) / cp;
      t -= dT;
      if (std::fabs(h - he) < 1e-7 || std::fabs(dT / t) < 1e-7) break;
    }
    T = t;
  }
  double lnT = std::log(T);
  double poly[5];
  poly[0] = 1.0; poly[1] = lnT; poly[2] = poly[1] * poly[1]; poly[3] = poly[1] * poly[2]; poly[4] = poly[2] * poly[2];
  psi = Wm / (R_GAS * T);
  rho = p * psi;
  double sv[64];
  for (int i = 0; i < S; ++i) { double dp = 0.; for (int j = 0; j < 5; ++j) dp += th.visc[i * 5 + j] * poly[j]; sv[i] = dp; }
  double mumix = 0.;
  for (int i = 0; i < S; ++i) {                            // Wilke (:111-151)
    double s2 = 0.;
    for (int j = 0; j < S; ++j) {
      double tmp = 1.0 + (sv[i] / sv[j]) * th.vc2[i * S + j];
      s2 += X[j] / SQRT8 * th.vc1[i * S + j] * (tmp * tmp);
    }
    mumix += X[i] * (sv[i] * sv[i]) / s2;
  }
  double sT = std::sqrt(T);
  mu = mumix * sT;
  double sc = 0., sic = 0.;
  for (int i = 0; i < S; ++i) {                            // (:172-206)
    double dp = 0.;
    for (int j = 0; j < 5; ++j) dp += th.cond[i * 5 + j] * poly[j];
    double lam = dp * sT;
    sc += X[i] * lam; sic += X[i] / lam;
  }
  alpha = 0.5 * (sc + 1.0 / sic) / cp_mix(th, T, y, ys);
  double powT = T * sT, rdp = rho / p;
  for (int i = 0; i < S; ++i) {                            // getMixDiffCoeffsMass (:208-255)
    if (X[i] + 1e-10 > 1.) { rhoD[i * os] = 0.; continue; }
    double s1 = 0., s2 = 0.;
    for (int j = 0; j < S; ++j) {
      if (i == j) continue;
      double tmp = 0.;
      for (int k = 0; k < 5; ++k) tmp += th.bdiff[(i * S + j) * 5 + k] * poly[k];
      double Dl = tmp * powT;
      s1 += X[j] / Dl;
      s2 += X[j] * th.W[j] / Dl;
    }
    s2 *= X[i] / (Wm - X[i] * th.W[i]);
    rhoD[i * os] = 1 / (s1 + s2) * rdp;
  }
  for (int i = 0; i < S; ++i) hai[i * os] = h_species(th, i, T);
}

// eeqn_calculate_energy_gradient (dfEEqn.cu:266-287 -> calculate_energy_gradient_kernel,
// dfThermo.cu:276-294): gradientEnergy slots of he get (h(T_c, Y_b) - h(T_c, Y_c)) * deltaCoeffs
void energy_gradient(const M& m) {
  const int* the = ia("ptype_he");
  double *T = d("T"), *Y = d("Y"), *bY = d("boundary_Y"), *eg = d("boundary_heGradient");
  #pragma omp parallel for schedule(static)
  for (int b = 0; b < m.B; ++b) {
    eg[b] = 0.0;
    if (the[m.slot_patch[b]] != GRAD_E) continue;
    int c = m.bfc[b];
    double hb = h_mix(g_th, T[c], bY + b, m.B), hc = h_mix(g_th, T[c], Y + c, m.C);
    eg[b] = (hb - hc) * m.bdc[b];
  }
}

// dfThermo::correctThermo (dfThermo.cu:572-671) / updateEnergy (from_T) (:567)
void thermo_correct(const M& m, bool from_T) {
  const int* tT = ia("ptype_T");
  const int C = m.C, B = m.B;
  double *T = d("T"), *he = d("he"), *p = d("p"), *Y = d("Y"), *psi = d("psi"), *rho = d("rho"), *mu = d("mu"),
         *alpha = d("alpha"), *rhoD = d("rhoD"), *hai = d("hai");
  double *bT = d("boundary_T"), *bhe = d("boundary_he"), *bp = d("boundary_p"), *bY = d("boundary_Y"),
         *bpsi = d("boundary_psi"), *brho = d("boundary_rho"), *bmu = d("boundary_mu"), *balpha = d("boundary_alpha"),
         *brhoD = d("boundary_rhoD"), *bhai = d("boundary_hai");
#pragma omp parallel for schedule(static)
  for (int c = 0; c < C; ++c)
    thermo_point(g_th, from_T, T[c], he[c], p[c], Y + c, C, psi[c], rho[c], mu[c], alpha[c], rhoD + c, hai + c, C);
#pragma omp parallel for schedule(static)
  for (int b = 0; b < B; ++b) {
    int t = tT[m.slot_patch[b]];
    if (t == EMPTY) continue;
    if (is_proc(t) && !m.primary[b]) {
      int c = m.bfc[b];
      bT[b] = T[c]; bhe[b] = he[c]; bpsi[b] = psi[c]; brho[b] = rho[c]; bmu[b] = mu[c]; balpha[b] = alpha[c];
      for (int s = 0; s < m.S; ++s) { brhoD[(long)s * B + b] = rhoD[(long)s * C + c]; bhai[(long)s * B + b] = hai[(long)s * C + c]; }
      continue;
    }
    thermo_point(g_th, from_T || fixes_value(t), bT[b], bhe[b], bp[b], bY + b, B, bpsi[b], brho[b], bmu[b], balpha[b],
                 brhoD + b, bhai + b, B);
  }
}

}  // namespace

extern "C" {

int orc_last_error(char* buf, int len) { std::snprintf(buf, len, "%s", g_err.c_str()); return (int)g_err.size(); }
void orc_clear() { D.clear(); I.clear(); }
void orc_set_d(const char* name, double* ptr) { D[name] = ptr; }
void orc_set_i(const char* name, int* ptr) { I[name] = ptr; }

int orc_set_thermo(int S, const double* W, const double* nasa, const double* visc, const double* cond, const double* bdiff) {
  g_th.S = S;
  g_th.W.assign(W, W + S);
  g_th.nasa.assign(nasa, nasa + 15 * S);
  g_th.visc.assign(visc, visc + 5 * S);
  g_th.cond.assign(cond, cond + 5 * S);
  g_th.bdiff.assign(bdiff, bdiff + 5 * S * S);
  g_th.vc1.resize(S * S); g_th.vc2.resize(S * S);
  for (int i = 0; i < S; ++i) for (int j = 0; j < S; ++j) {   // init_const_coeff_ptr (dfThermo.cu:22-52)
    g_th.vc1[i * S + j] = std::pow((1 + W[i] / W[j]), -0.5);
    g_th.vc2[i * S + j] = std::pow(W[j] / W[i], 0.25);
  }
  return 0;
}

#define ORC_CALL(body) try { M m = mesh(); body; return 0; } catch (std::exception& e) { g_err = e.what(); return 1; }

int orc_rho_eqn() { ORC_CALL(rho_eqn(m)) }
int orc_u_assemble() { ORC_CALL(u_eqn_assemble(m)) }
int orc_u_hbya() { ORC_CALL(u_hbya(m)) }
int orc_p_assemble() { ORC_CALL(p_eqn_assemble(m)) }
int orc_p_post() { ORC_CALL(p_eqn_post(m)) }
int orc_y_prep() { ORC_CALL(y_prep(m)) }
int orc_y_assemble() { ORC_CALL(y_assemble(m)) }
int orc_y_inert() { ORC_CALL(y_inert(m)) }
int orc_e_assemble() { ORC_CALL(e_assemble(m)) }
int orc_thermo_correct(int from_T) { ORC_CALL(thermo_correct(m, from_T != 0)) }
int orc_energy_gradient() { ORC_CALL(energy_gradient(m)) }
// convection weights of div(phi,Yi_h) -> "conv_w" / "boundary_conv_w" (start of YEqn, reused by EEqn)
int orc_conv_weights() { ORC_CALL(conv_weights(m)) }
// inspection: cubic's explicit flux correction of hDiffCorrFlux -> "out_cubic_flux" [F], "out_boundary_cubic_flux" [B];
// the div(phi,K) weights -> "out_K_w" [F], "out_boundary_K_w" [B]
int orc_cubic_flux() { ORC_CALL(cubic_flux(m, ia("ptype_calculated"), d("hDiffCorrFlux"), d("boundary_hDiffCorrFlux"),
                                           d("out_cubic_flux"), d("out_boundary_cubic_flux"))) }
int orc_k_weights() { ORC_CALL(k_weights(m, d("out_K_w"), d("out_boundary_K_w"))) }
// inspection: the div(phi,U) limitedLinearV weights -> "out_U_w" [F], "out_boundary_U_w" [B]
int orc_u_weights() {
  ORC_CALL({
    std::vector<double> g(9L * m.C);
    grad_vector(m, ia("ptype_U"), d("U"), d("boundary_U"), g.data());
    u_weights(m, ia("ptype_U"), d("U"), g.data(), d("phi"), d("boundary_phi"), d("out_U_w"), d("out_boundary_U_w"));
  })
}
int orc_correct_bc(const char* field, const char* bfield, const char* ptype, int ncomp) {
  const Mix mx = mix_for(field);
  ORC_CALL(correct_bc_vec(m, ia(ptype), d(field), d(bfield), ncomp, &mx))
}
int orc_grad_scalar(const char* field, const char* bfield, const char* ptype, const char* out, const char* bout) {
  ORC_CALL(grad_scalar(m, ia(ptype), d(field), d(bfield), d(out), bout ? d(bout) : nullptr))
}
int orc_thermo_points(int n, int fixT, double* T, double* he, const double* p, const double* Y, double* psi, double* rho,
                      double* mu, double* alpha, double* rhoD, double* hai) {
  try {
#pragma omp parallel for schedule(static)
    for (int c = 0; c < n; ++c)
      thermo_point(g_th, fixT != 0, T[c], he[c], p[c], Y + c, n, psi[c], rho[c], mu[c], alpha[c], rhoD + c, hai + c, n);
    return 0;
  } catch (std::exception& e) { g_err = e.what(); return 1; }
}

}  // extern "C"
