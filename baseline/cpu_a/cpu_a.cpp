// cpu_a.cpp -- CPU-A: the build's own OpenMP C++ CPU implementation of one
// dfLowMachFoam outer iteration (applications/solvers/dfLowMachFoam/dfLowMachFoam.C:249-531 with
// nOuterCorrectors = 1) behind the same C ABI as the HIP path (include/dfmi.h). It is the CPU baseline
// bench.py times beside the GPU step, on all the host cores it is given. It is NOT the product:
// nothing under deepflame-dev_amd/ loads it, and it ships as its own library (libdfmi_cpu_a.so).
//
//  * FV assembly, boundary correction and thermo/transport: the restatement in oracle/df_oracle.cpp
//    (linked in), whose face loops run as OpenMP per-cell gathers; its LDU systems are the ones the GPU
//    path assembles bit for bit (tests/test_gpu_parity.py).
//  * linear solves: Jacobi-preconditioned BiCGStab for U, Y_i and he, and CG preconditioned by the
//    aggregation-AMG V-cycle for p -- the GPU path's methods, parameters and stopping rule
//    (||b - A x||_2 <= tol ||b - A x0||_2, AmgX RELATIVE_INI), row-parallel over ELL operators [W][C];
//    the AMG hierarchy is built by the same code as the GPU's (csrc/amg_graph.h), the V-cycle in fp64.
//  * chemistry: ROS3 with the generated kinetics (csrc/chem_gen_*.inc), the GPU path's step control,
//    Cantera setState_TPY reactor state and RR scaled by the step-start density (chem.hip), one cell
//    per OpenMP iteration (dynamic schedule: stiff cells cost 10-100x the others).
// Single rank (no processor patches); DNN chemistry, renumbering and kernel timers are GPU-path only.
// Also runs BASELINE configs 1 (dfmi_zero_d_step) and 2 (the 1D flame's mixed outlet) for bench.py.
#include "../../include/dfmi.h"
#include "../../deepflame-dev_amd/csrc/amg_graph.h"

#include <omp.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <exception>
#include <functional>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#define DFMI_HD   // the generated kinetics run on the host here
#define DFMI_SCHED_FENCE()   // scheduling barrier of the device build only
#define DFMI_CONTRACT() do {} while (0)   // FMA contraction of the device build only
#define DFMI_RCP(x) (1.0 / (x))           // the device build's refined hardware reciprocal
#pragma GCC diagnostic push
#pragma GCC diagnostic ignored "-Wunused-variable"
#include "../../deepflame-dev_amd/csrc/chem_gen_burke9.inc"
#include "../../deepflame-dev_amd/csrc/chem_gen_es80.inc"
#pragma GCC diagnostic pop

// the oracle restatement's stages (oracle/df_oracle.cpp)
extern "C" {
void orc_clear();
void orc_set_d(const char* name, double* ptr);
void orc_set_i(const char* name, int* ptr);
int orc_last_error(char* buf, int len);
int orc_set_thermo(int S, const double* W, const double* nasa, const double* visc, const double* cond, const double* bdiff);
int orc_rho_eqn();
int orc_u_assemble();
int orc_u_hbya();
int orc_p_assemble();
int orc_p_post();
int orc_y_prep();
int orc_y_assemble();
int orc_y_inert();
int orc_e_assemble();
int orc_thermo_correct(int from_T);
int orc_energy_gradient();
int orc_correct_bc(const char* field, const char* bfield, const char* ptype, int ncomp);
int orc_conv_weights();
}

struct dfmi_ctx;

namespace {

enum BC { ZG = 0, FV = 1, COUPLED = 2, EMPTY = 3, GRAD_E = 4, CALC = 5, CYCLIC = 6, PROC = 7, EXTRAP = 8,
          FIX_E = 9, PROC_CYC = 10, WAVE = 11, IN_OUT = 12 };
inline bool is_coupled(int t) { return t == CYCLIC || t == PROC || t == PROC_CYC || t == COUPLED; }

std::string g_err;
struct Error : std::runtime_error { using std::runtime_error::runtime_error; };
#define CHECK(c, msg) do { if (!(c)) throw Error(std::string("dfmi (CPU-A): ") + (msg)); } while (0)

void orc(int rc, const char* what) {
  if (rc == 0) return;
  char buf[2048];
  orc_last_error(buf, sizeof buf);
  throw Error(std::string("dfmi (CPU-A): ") + what + ": " + buf);
}

struct Field { std::vector<double> v; long n = 0; int ncomp = 1; };
struct SolverCfg { int max_iter; double tol, abs_tol; int precond; };   // precond 0 Jacobi, 1 AMG
struct Stats { int iters = 0; double res0 = 0, res = 0; double work = 0; };

struct Level {                       // AMG level: ELL [W][n] + diagonal, work vectors
  int n = 0, W = 0;
  std::vector<int> col, agg, mstart, members, gstart, gsrc;
  std::vector<double> val, D, b, x, r, xo;
};

struct Ctx {
  int C = 0, Ctot = 0, F = 0, B = 0, P = 0, S = 0, inert = -1;
  double rdt = 0;
  bool have_sizes = false, have_topo = false, have_geom = false, have_bgeom = false;
  std::vector<int> psize, pkind, cyc_nbr, own, nei, bfc, poff, slot_patch, prim, partner, dims, inert_v;
  std::map<std::string, std::vector<int>> ptype;        // per patch, also registered as "ptype_<f>"
  std::map<std::string, Field> fields;                  // user-visible fields (SoA [ncomp][n])
  std::map<std::string, std::vector<double>> work;      // oracle inputs/outputs that are not fields
  std::vector<double> rdt_v;
  // schemes (dfmi_set_scheme; the oracle's "schemes" / "scheme_k" layout)
  std::vector<int> schemes{0, 1, 1, 1};
  std::vector<double> scheme_k{1.0, 1.0, 1.0};
  // thermo
  std::vector<double> W, nasa, visc, cond, bdiff;
  // solvers
  std::map<std::string, SolverCfg> solver;
  std::map<std::string, Stats> stats;
  int ellW = 0;
  std::vector<int> ecol;          // [W][C]
  std::vector<long> esrc;         // [W][C]: f upper, F + f lower, 2F + b coupled slot, -1 padding
  std::vector<int> cbStart, cbSlot;
  std::vector<Level> amg;
  bool amg_ready = false;
  // chemistry
  int mode = 0, max_steps = 100000, R = 0, generated = 0;
  double rtol = 1e-6, atol = 1e-10, Tmin = 0.0;
  std::vector<int> idata, irs;
  std::vector<double> dd;

  double* f(const std::string& n) {
    auto it = fields.find(n);
    CHECK(it != fields.end(), "unknown field '" + n + "'");
    return it->second.v.data();
  }
  double* w(const std::string& n) { return work.at(n).data(); }
};

template <class FN> int guard(FN&& fn) {
  try { fn(); return 0; } catch (std::exception& e) { g_err = e.what(); return 1; }
}

// ---------------------------------------------------------------- setup
void alloc(Ctx& x, const std::string& n, long len, int ncomp) {
  Field& f = x.fields[n];
  f.n = len; f.ncomp = ncomp;
  f.v.assign((size_t)len * ncomp, 0.0);
}

void allocate_fields(Ctx& x) {
  const long C = x.C, B = x.B, F = x.F;
  const int S = x.S;
  for (auto n : {"rho", "rho_old", "p", "p_old", "he", "T", "K", "K_old", "psi", "mu", "alpha", "dpdt", "rAU",
                 "diffAlphaD", "psip0"}) { alloc(x, n, C, 1); alloc(x, std::string("boundary_") + n, B, 1); }
  for (auto n : {"U", "U_old", "HbyA", "hDiffCorrFlux", "sumYDiffError"}) { alloc(x, n, C, 3); alloc(x, std::string("boundary_") + n, B, 3); }
  for (auto n : {"Y", "rhoD", "hai", "RR"}) { alloc(x, n, C, S); alloc(x, std::string("boundary_") + n, B, S); }
  for (auto n : {"phi", "phi_old", "phiUc", "rhorAUf", "phiHbyA"}) { alloc(x, n, F, 1); alloc(x, std::string("boundary_") + n, B, 1); }
  alloc(x, "boundary_heGradient", B, 1);
  alloc(x, "boundary_p_vf", B, 1);
  alloc(x, "boundary_p_gamma", B, 1);
  alloc(x, "boundary_U_ref", B, 3);
  alloc(x, "boundary_p_ref", B, 1);
  alloc(x, "boundary_Y_ref", B, S);
  alloc(x, "boundary_K_ref", B, 1);
  alloc(x, "chem_stats", C, 3);
  alloc(x, "Qdot", C, 1);   // heat release -sum_i hc_i RR_i (dfChemistryModel.C:771)
  const long ns = std::max(S, 3);
  auto wk = [&](const std::string& n, long len) { x.work[n].assign(std::max(len, 1L), 0.0); };
  wk("out_lower", (long)S * F); wk("out_upper", (long)S * F); wk("out_diag", (long)S * C);
  wk("out_source", ns * C); wk("out_source_solve", 3 * C);
  wk("out_internal_coeffs", ns * B); wk("out_boundary_coeffs", ns * B);
  wk("out_rhorAUf", F); wk("out_boundary_rhorAUf", B); wk("out_phiHbyA", F); wk("out_boundary_phiHbyA", B);
  for (auto n : {"lower", "upper"}) { wk(std::string("ueqn_") + n, F); wk(std::string("peqn_") + n, F); }
  wk("ueqn_source", 3 * C); wk("ueqn_internal_coeffs", 3 * B); wk("ueqn_boundary_coeffs", 3 * B);
  wk("peqn_internal_coeffs", B); wk("peqn_boundary_coeffs", B); wk("peqn_phiHbyA", F); wk("peqn_boundary_phiHbyA", B);
  wk("conv_w", F); wk("boundary_conv_w", B);   // div(phi,Yi_h) weights (start of YEqn, reused by EEqn)
  if (!x.work.count("boundary_delta")) wk("boundary_delta", 3 * B);
  for (auto e : {"U", "Y", "E"}) if (!x.solver.count(e)) x.solver[e] = SolverCfg{20, 1e-5, 0.0, 0};   // amgxUOptions
  if (!x.solver.count("p")) x.solver["p"] = SolverCfg{1000, 1e-5, 0.0, 1};                            // amgxpOptions
}

// Term-sensitivity study knobs (DFMI_CPUA_STUDY, comma list; unset in every product / bench / test run):
// no_diffAlphaD, no_hDiffCorrFlux, no_dpdt drop that EEqn term; ddtcorr=<s> scales pEqn's ddtCorr flux
// (pEqn.H:21-25). scripts/tgv2d_terms.py tabulates each one's effect on test/corrtest.cpp:52-56.
bool study(const char* knob) {
  const char* e = std::getenv("DFMI_CPUA_STUDY");
  return e && std::strstr(e, knob) != nullptr;
}
// "<name>=<s>": scale a term by s (1 when absent)
double study_scale(const char* name) {
  const char* e = std::getenv("DFMI_CPUA_STUDY");
  const std::string key = std::string(name) + "=";
  const char* at = e ? std::strstr(e, key.c_str()) : nullptr;
  return at ? std::atof(at + key.size()) : 1.0;
}
void scale_field(Ctx& x, const char* name, long n, double s) {
  if (s == 1.0) return;
  double* v = x.f(name);
  for (long i = 0; i < n; ++i) v[i] *= s;
}
double g_ddtcorr_scale = 1.0;

// register every array with the oracle restatement (its registry is process-global)
void bind(Ctx& x) {
  CHECK(x.have_bgeom, "mesh not fully initialised");
  CHECK(!x.W.empty(), "thermo coefficients not set");
  orc_clear();
  x.dims = {x.C, x.F, x.B, x.P, x.S};
  x.inert_v = {x.inert};
  orc_set_i("dims", x.dims.data());
  orc_set_i("owner", x.own.data()); orc_set_i("neighbour", x.nei.data());
  orc_set_i("patch_size", x.psize.data()); orc_set_i("cyclic_neighbor", x.cyc_nbr.data());
  orc_set_i("boundary_face_cell", x.bfc.data()); orc_set_i("patch_kind", x.pkind.data());
  orc_set_i("inert_index", x.inert_v.data());
  for (auto& kv : x.ptype) orc_set_i(("ptype_" + kv.first).c_str(), kv.second.data());
  x.rdt_v = {x.rdt};
  orc_set_d("rdelta_t", x.rdt_v.data());
  orc_set_i("schemes", x.schemes.data());
  orc_set_d("scheme_k", x.scheme_k.data());
  for (auto& kv : x.fields) orc_set_d(kv.first.c_str(), kv.second.v.data());
  for (auto& kv : x.work) orc_set_d(kv.first.c_str(), kv.second.data());
  orc(orc_set_thermo(x.S, x.W.data(), x.nasa.data(), x.visc.data(), x.cond.data(), x.bdiff.data()), "thermo");
  if (const char* e = std::getenv("DFMI_CPUA_STUDY"); e && std::strstr(e, "ddtcorr=")) {
    g_ddtcorr_scale = std::atof(std::strstr(e, "ddtcorr=") + 8);
    orc_set_d("study_ddtcorr_scale", &g_ddtcorr_scale);
  }
}

void require_ready(Ctx& x) {
  CHECK(x.have_sizes && x.have_topo && x.have_geom && x.have_bgeom, "mesh not fully initialised");
  for (auto f : {"U", "p", "he", "K", "Y", "T", "rho"}) CHECK(x.ptype.count(f), std::string("patch types of '") + f + "' not set");
  CHECK(x.inert >= 0, "inert species index not set");
  bind(x);
}

// solver rows: per cell its faces in increasing index (neighbour side: lower, owner side: upper), then
// its coupled boundary slots; the same entry order the GPU's ELL uses (linsolve.hip)
void build_rows(Ctx& x) {
  const int C = x.C, F = x.F, B = x.B;
  std::vector<std::vector<long>> ent(C);
  std::vector<std::vector<int>> ecol(C);
  for (int f = 0; f < F; ++f) {
    ent[x.nei[f]].push_back(F + (long)f); ecol[x.nei[f]].push_back(x.own[f]);
  }
  for (int f = 0; f < F; ++f) { ent[x.own[f]].push_back(f); ecol[x.own[f]].push_back(x.nei[f]); }
  for (int b = 0; b < B; ++b) {
    if (!x.prim[b] || x.partner[b] < 0) continue;
    const int c = x.bfc[b];
    ent[c].push_back(2L * F + b); ecol[c].push_back(x.partner[b]);
  }
  int W = 1;
  for (int c = 0; c < C; ++c) W = std::max(W, (int)ent[c].size());
  x.ellW = W;
  x.ecol.assign((size_t)W * C, 0);
  x.esrc.assign((size_t)W * C, -1);
  for (int c = 0; c < C; ++c)
    for (int k = 0; k < W; ++k) {
      const bool have = k < (int)ent[c].size();
      x.ecol[(size_t)k * C + c] = have ? ecol[c][k] : c;
      x.esrc[(size_t)k * C + c] = have ? ent[c][k] : -1;
    }
  x.cbStart.assign(C + 1, 0);
  for (int b = 0; b < B; ++b) if (x.prim[b]) x.cbStart[x.bfc[b] + 1]++;
  for (int c = 0; c < C; ++c) x.cbStart[c + 1] += x.cbStart[c];
  x.cbSlot.assign(std::max(x.cbStart[C], 1), 0);
  std::vector<int> pos(x.cbStart.begin(), x.cbStart.end() - 1);
  for (int b = 0; b < B; ++b) if (x.prim[b]) x.cbSlot[pos[x.bfc[b]]++] = b;
}

// ---------------------------------------------------------------- linear algebra
struct Sys { const double* val; const double* D; const int* col; int W, n; };

inline void spmv(const Sys& A, const double* xv, double* y) {
#pragma omp parallel for schedule(static)
  for (int c = 0; c < A.n; ++c) {
    double a = A.D[c] * xv[c];
    for (int k = 0; k < A.W; ++k) a += A.val[(size_t)k * A.n + c] * xv[A.col[(size_t)k * A.n + c]];
    y[c] = a;
  }
}
inline double dot(int n, const double* a, const double* b) {
  double s = 0.0;
#pragma omp parallel for reduction(+ : s) schedule(static)
  for (int i = 0; i < n; ++i) s += a[i] * b[i];
  return s;
}

// LDU (+ boundary coefficients of the field's patch types) -> ELL values, diag + internalCoeffs,
// source + boundaryCoeffs (fvMatrix::addBoundaryDiag / addBoundarySource)
void fold(Ctx& x, const double* lower, const double* upper, const double* diag, const double* source, const double* ic,
          const double* bc, const std::vector<int>& tp, std::vector<double>& val, std::vector<double>& D,
          std::vector<double>& rhs) {
  const int C = x.C, F = x.F, W = x.ellW;
  val.resize((size_t)W * C); D.resize(C); rhs.resize(C);
#pragma omp parallel for schedule(static)
  for (int c = 0; c < C; ++c) {
    for (int k = 0; k < W; ++k) {
      const long s = x.esrc[(size_t)k * C + c];
      double v = 0.0;
      if (s >= 0 && s < F) v = upper[s];
      else if (s >= F && s < 2L * F) v = lower[s - F];
      else if (s >= 2L * F) {
        const int b = (int)(s - 2L * F);
        v = tp[x.slot_patch[b]] == EMPTY ? 0.0 : -bc[b];
      }
      val[(size_t)k * C + c] = v;
    }
    double d = diag[c], r = source[c];
    for (int e = x.cbStart[c]; e < x.cbStart[c + 1]; ++e) {
      const int b = x.cbSlot[e];
      const int t = tp[x.slot_patch[b]];
      if (t == EMPTY) continue;
      d += ic[b];
      if (!is_coupled(t)) r += bc[b];
    }
    D[c] = d; rhs[c] = r;
  }
}

// Jacobi-preconditioned BiCGStab (right preconditioning), x in/out
Stats bicgstab(const Sys& A, const double* b, double* xv, const SolverCfg& cfg) {
  const int n = A.n;
  std::vector<double> r(n), rh(n), p(n, 0.0), v(n, 0.0), y(n), s(n), z(n), t(n);
  spmv(A, xv, r.data());
#pragma omp parallel for schedule(static)
  for (int i = 0; i < n; ++i) { r[i] = b[i] - r[i]; rh[i] = r[i]; }
  Stats st;
  st.res0 = std::sqrt(dot(n, r.data(), r.data()));
  double res = st.res0, rho = 1.0, alpha = 1.0, omega = 1.0;
  int it = 0;
  while (!(res <= cfg.tol * st.res0 || res <= cfg.abs_tol || it >= cfg.max_iter)) {
    const double rho_n = dot(n, rh.data(), r.data());
    if (rho_n == 0.0) break;
    const double beta = (rho_n / rho) * (alpha / omega);
    rho = rho_n;
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) { p[i] = r[i] + beta * (p[i] - omega * v[i]); y[i] = p[i] / A.D[i]; }
    spmv(A, y.data(), v.data());
    const double rv = dot(n, rh.data(), v.data());
    if (rv == 0.0) break;
    alpha = rho / rv;
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) { s[i] = r[i] - alpha * v[i]; z[i] = s[i] / A.D[i]; }
    spmv(A, z.data(), t.data());
    double tt = 0.0, ts = 0.0;
#pragma omp parallel for reduction(+ : tt, ts) schedule(static)
    for (int i = 0; i < n; ++i) { tt += t[i] * t[i]; ts += t[i] * s[i]; }
    omega = tt > 0.0 ? ts / tt : 0.0;
    double rr = 0.0;
#pragma omp parallel for reduction(+ : rr) schedule(static)
    for (int i = 0; i < n; ++i) {
      xv[i] += alpha * y[i] + omega * z[i];
      r[i] = s[i] - omega * t[i];
      rr += r[i] * r[i];
    }
    res = std::sqrt(rr);
    ++it;
    if (omega == 0.0) break;
  }
  st.iters = it; st.res = st.res0 > 0 ? res / st.res0 : 0.0; st.work = it;
  return st;
}

// ---- AMG (hierarchy from csrc/amg_graph.h, V-cycle as amg.hip's, fp64)
constexpr double AMG_OMEGA = 0.9, AMG_OVERCORR = 1.4;
constexpr int AMG_COARSE_SWEEPS = 6, AMG_COARSEST = 512;

void amg_setup(Ctx& x) {
  x.amg.clear();
  const int C = x.C;
  const std::vector<double>& mag = x.work.at("mag_sf");
  const std::vector<double>& dcf = x.work.at("delta_coeffs");
  const std::vector<double>& bmag = x.work.at("boundary_mag_sf");
  const std::vector<double>& bdc = x.work.at("boundary_delta_coeffs");
  std::vector<double> fs(x.F);
  for (int f = 0; f < x.F; ++f) fs[f] = mag[f] * dcf[f];
  std::vector<int> co, cn;
  std::vector<double> cs;
  for (int p = 0; p < x.P; ++p) {
    if (x.pkind[p] != 1) continue;
    const int q = x.cyc_nbr[p];
    for (int i = 0; i < x.psize[p]; ++i) {
      const int b = x.poff[p] + i;
      co.push_back(x.bfc[b]); cn.push_back(x.bfc[x.poff[q] + i]); cs.push_back(bmag[b] * bdc[b]);
    }
  }
  dfmi::Graph g = dfmi::strength_graph(C, x.own, x.nei, fs, co, cn, cs);
  x.amg.emplace_back();
  x.amg[0].n = C; x.amg[0].W = x.ellW; x.amg[0].col = x.ecol;
  auto too_big = [&](const Level& l) { return l.n > AMG_COARSEST || (size_t)l.n * l.W > 6144; };
  while (too_big(x.amg.back())) {
    Level& f = x.amg.back();
    dfmi::AmgCoarse k = dfmi::amg_coarsen(f.col, f.W, f.n, g);
    f.agg = std::move(k.agg); f.mstart = std::move(k.mstart); f.members = std::move(k.members);
    f.gstart = std::move(k.gstart); f.gsrc = std::move(k.gsrc);
    Level c;
    c.n = k.nc; c.W = k.Wc; c.col = std::move(k.ccol);
    const bool stalled = c.n * 2 > f.n;
    g = std::move(k.cg);
    x.amg.push_back(std::move(c));
    if (stalled) break;
  }
  for (size_t l = 0; l < x.amg.size(); ++l) {
    Level& v = x.amg[l];
    if (l > 0) { v.val.resize((size_t)v.W * v.n); v.D.resize(v.n); v.b.resize(v.n); }
    v.x.resize(v.n); v.r.resize(v.n); v.xo.resize(v.n);
  }
  x.amg_ready = true;
}

void amg_galerkin(Ctx& x, const double* val0, const double* D0) {
  for (size_t l = 0; l + 1 < x.amg.size(); ++l) {
    Level& f = x.amg[l];
    Level& c = x.amg[l + 1];
    const double* fv = l == 0 ? val0 : f.val.data();
    const double* fD = l == 0 ? D0 : f.D.data();
    const int slots = c.W + 1, nc = c.n;
#pragma omp parallel for schedule(static)
    for (int I = 0; I < nc; ++I)
      for (int s = 0; s < slots; ++s) {
        double a = 0.0;
        for (int e = f.gstart[(size_t)s * nc + I]; e < f.gstart[(size_t)s * nc + I + 1]; ++e) {
          const int src = f.gsrc[e];
          a += src >= 0 ? fv[src] : fD[-src - 1];
        }
        if (s < slots - 1) c.val[(size_t)s * nc + I] = a;
        else c.D[I] = a;
      }
  }
}

void amg_apply(Ctx& x, const double* val0, const double* D0, const double* r0, double* z) {
  const int L = (int)x.amg.size();
  auto VAL = [&](int l) { return l == 0 ? val0 : x.amg[l].val.data(); };
  auto DD = [&](int l) { return l == 0 ? D0 : x.amg[l].D.data(); };
  const double om = AMG_OMEGA, sc = AMG_OVERCORR;
  for (int l = 0; l + 1 < L; ++l) {        // down: one sweep from zero + residual, restrict
    Level& f = x.amg[l];
    const double *val = VAL(l), *D = DD(l), *b = l == 0 ? r0 : f.b.data();
    const int n = f.n, W = f.W;
#pragma omp parallel for schedule(static)
    for (int c = 0; c < n; ++c) f.x[c] = om * b[c] / D[c];
#pragma omp parallel for schedule(static)
    for (int c = 0; c < n; ++c) {
      double y = D[c] * f.x[c];
      for (int k = 0; k < W; ++k) {
        const int j = f.col[(size_t)k * n + c];
        y += val[(size_t)k * n + c] * f.x[j];
      }
      f.r[c] = b[c] - y;
    }
    Level& cl = x.amg[l + 1];
#pragma omp parallel for schedule(static)
    for (int I = 0; I < cl.n; ++I) {
      double a = 0.0;
      for (int e = f.mstart[I]; e < f.mstart[I + 1]; ++e) a += f.r[f.members[e]];
      cl.b[I] = a;
    }
  }
  {                                         // coarsest: weighted-Jacobi sweeps from zero
    Level& c = x.amg[L - 1];
    const double *val = VAL(L - 1), *D = DD(L - 1), *b = L == 1 ? r0 : c.b.data();
    double* out = L == 1 ? z : c.x.data();
    const int n = c.n, W = c.W;
    std::vector<double> cur(n), nxt(n);
    for (int i = 0; i < n; ++i) cur[i] = om * b[i] / D[i];
    for (int s = 1; s < AMG_COARSE_SWEEPS; ++s) {
#pragma omp parallel for schedule(static) if (n > 4096)
      for (int i = 0; i < n; ++i) {
        double y = D[i] * cur[i];
        for (int k = 0; k < W; ++k) y += val[(size_t)k * n + i] * cur[c.col[(size_t)k * n + i]];
        nxt[i] = cur[i] + om * (b[i] - y) / D[i];
      }
      cur.swap(nxt);
    }
    for (int i = 0; i < n; ++i) out[i] = cur[i];
  }
  for (int l = L - 2; l >= 0; --l) {        // up: prolongate the scaled coarse correction + one sweep
    Level& f = x.amg[l];
    const Level& cl = x.amg[l + 1];
    const double *val = VAL(l), *D = DD(l), *b = l == 0 ? r0 : f.b.data();
    double* out = l == 0 ? z : f.xo.data();
    const int n = f.n, W = f.W;
#pragma omp parallel for schedule(static)
    for (int c = 0; c < n; ++c) {
      const double yc = f.x[c] + sc * cl.x[f.agg[c]];
      double ay = D[c] * yc;
      for (int k = 0; k < W; ++k) {
        const int j = f.col[(size_t)k * n + c];
        ay += val[(size_t)k * n + c] * (f.x[j] + sc * cl.x[f.agg[j]]);
      }
      out[c] = yc + om * (b[c] - ay) / D[c];
    }
    if (l > 0) f.x.swap(f.xo);
  }
}

// CG preconditioned by Jacobi or the AMG V-cycle, x in/out
Stats pcg(Ctx& x, const Sys& A, const double* b, double* xv, const SolverCfg& cfg) {
  const int n = A.n;
  std::vector<double> r(n), z(n), p(n), q(n);
  spmv(A, xv, r.data());
#pragma omp parallel for schedule(static)
  for (int i = 0; i < n; ++i) r[i] = b[i] - r[i];
  Stats st;
  st.res0 = std::sqrt(dot(n, r.data(), r.data()));
  double res = st.res0;
  const bool amg = cfg.precond == 1;
  if (amg) {
    if (!x.amg_ready) amg_setup(x);
    amg_galerkin(x, A.val, A.D);
  }
  auto prec = [&]() {
    if (amg) amg_apply(x, A.val, A.D, r.data(), z.data());
    else {
#pragma omp parallel for schedule(static)
      for (int i = 0; i < n; ++i) z[i] = r[i] / A.D[i];
    }
  };
  int it = 0;
  double rz = 0.0;
  while (!(res <= cfg.tol * st.res0 || res <= cfg.abs_tol || it >= cfg.max_iter)) {
    prec();
    const double rzn = dot(n, r.data(), z.data());
    if (rzn == 0.0) break;
    const double beta = it == 0 ? 0.0 : rzn / rz;
    rz = rzn;
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) p[i] = z[i] + beta * p[i];
    spmv(A, p.data(), q.data());
    const double pq = dot(n, p.data(), q.data());
    if (pq == 0.0) break;
    const double alpha = rz / pq;
    double rr = 0.0;
#pragma omp parallel for reduction(+ : rr) schedule(static)
    for (int i = 0; i < n; ++i) {
      xv[i] += alpha * p[i];
      r[i] -= alpha * q[i];
      rr += r[i] * r[i];
    }
    res = std::sqrt(rr);
    ++it;
  }
  st.iters = it; st.res = st.res0 > 0 ? res / st.res0 : 0.0; st.work = it;
  return st;
}

void record(Ctx& x, const std::string& e, const Stats& s, bool first) {
  Stats& t = x.stats[e];
  const double w = t.work;
  if (first || s.iters > t.iters) { t.iters = s.iters; t.res0 = s.res0; t.res = s.res; }
  t.work = w + s.work;
}

// solve one LDU system of field `ptype` into xv (initial guess: its current values)
void solve(Ctx& x, const std::string& eqn, const double* lower, const double* upper, const double* diag,
           const double* source, const double* ic, const double* bc, const std::string& ptype, double* xv, bool first) {
  std::vector<double> val, D, rhs;
  fold(x, lower, upper, diag, source, ic, bc, x.ptype.at(ptype), val, D, rhs);
  const Sys A{val.data(), D.data(), x.ecol.data(), x.ellW, x.C};
  const SolverCfg& cfg = x.solver.at(eqn);
  const Stats s = cfg.precond == 1 || eqn == "p" ? pcg(x, A, rhs.data(), xv, cfg) : bicgstab(A, rhs.data(), xv, cfg);
  record(x, eqn, s, first);
}

// ---------------------------------------------------------------- chemistry (chem.hip k_chem_gen, host)
constexpr double RU = 8314.46261815324;

unsigned long long fnv(unsigned long long h, const void* p, size_t n) {
  const unsigned char* b = static_cast<const unsigned char*>(p);
  for (size_t i = 0; i < n; ++i) { h ^= b[i]; h *= 0x100000001b3ull; }
  return h;
}

// hc_i = Hf298_i / W_i (dfChemistryModel.C:335-338), the expression of thermo.hip heat_of_formation_per_mass
std::vector<double> hf298_per_mass(const Ctx& x) {
  std::vector<double> hc(x.S);
  const double T = 298.15, T2 = T * T, T3 = T2 * T, T4 = T3 * T, rT = 1.0 / T;
  for (int i = 0; i < x.S; ++i) {
    const double* row = x.nasa.data() + 15 * i;
    const double* a = T <= row[0] ? row + 8 : row + 1;
    const double ct0 = a[0], ct1 = a[1] * T, ct2 = a[2] * T2, ct3 = a[3] * T3, ct4 = a[4] * T4;
    const double h_RT = ct0 + 0.5 * ct1 + (1.0 / 3.0) * ct2 + 0.25 * ct3 + 0.2 * ct4 + a[5] * rT;
    hc[i] = h_RT * RU * T / x.W[i];
  }
  return hc;
}

template <class G>
int chem_cells(Ctx& x, double dt, const double* rho_rr) {
  constexpr int S = G::S, SA = G::SA;   // active species: the integrated state (chem.hip k_chem_gen)
  constexpr double g = 0.43586652150845899941601945119356;
  constexpr double c21 = -0.10156171083877702091975600115545e1, c31 = 0.40759956452537699824805835358067e1,
                   c32 = 0.92076794298330791242156818474003e1;
  constexpr double m2 = 0.61697947043828245592553615689730e1, m3 = -0.42772256543218573326238373806514;
  constexpr double e1 = 0.5, e2 = -0.29079558716805469821718236208017e1, e3 = 0.22354069897811569627360909276199;
  const long n = x.C;
  const double *Tf = x.f("T"), *pf = x.f("p"), *Yf = x.f("Y");
  double *RR = x.f("RR"), *stats = x.f("chem_stats"), *Qdot = x.f("Qdot");
  const double rtol = x.rtol, atol = x.atol, Tmin = x.Tmin;
  const std::vector<double> hc = hf298_per_mass(x);
  const int max_steps = x.max_steps;
  int fail = 0;
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : fail)
  for (long c = 0; c < n; ++c) {
    const double T = Tf[c];
    double Y0[S], y[S], sc[S];
    double ys = 0.0, sw = 0.0;   // setState_TPY: clipped, normalised Y; rho = p W / (R T)
    for (int i = 0; i < S; ++i) { Y0[i] = Yf[(long)i * n + c]; ys += std::fmax(Y0[i], 0.0); }
    const double iys = 1.0 / ys;
    for (int i = 0; i < S; ++i) sw += std::fmax(Y0[i], 0.0) * iys / G::W[i];
    const double rho = pf[c] / (sw * RU * T);
    for (int i = 0; i < S; ++i) { y[i] = rho * (std::fmax(Y0[i], 0.0) * iys) / G::W[i]; sc[i] = atol * rho * G::RW[i]; }
    int steps = 0, rejects = 0;
    double hnext = 0.0;
    if (T >= Tmin) {
      double k[G::NK];
      G::consts(T, k);
      const double hp = stats[2 * n + c];
      double t = 0.0, h = hp > 0.0 ? std::fmin(dt, hp) : dt;
      while (t < dt) {
        if (steps + rejects >= max_steps) { steps = -1; break; }
        if (t + h > dt) h = dt - t;
        const double hg = h * g, rh = 1.0 / h;
        double f0[SA], A[SA * SA];
        for (int e = 0; e < SA * SA; ++e) A[e] = 0.0;
        G::wdot_jac(T, k, y, f0, A);
        for (int e = 0; e < SA * SA; ++e) A[e] = (e % (SA + 1) == 0 ? 1.0 : 0.0) - hg * A[e];
        bool ok = G::factor(A);
        double err = 0.0, yn[SA];
        if (ok) {
          double k1[SA], k2[SA], k3[SA], y2[S], f2[SA];
          for (int a = 0; a < SA; ++a) k1[a] = hg * f0[a];
          G::solve(A, k1);
          for (int i = 0; i < S; ++i) y2[i] = y[i];
          for (int a = 0; a < SA; ++a) y2[G::ACT[a]] = y[G::ACT[a]] + k1[a];
          G::wdot(T, k, y2, f2);
          for (int a = 0; a < SA; ++a) k2[a] = hg * (f2[a] + c21 * rh * k1[a]);
          G::solve(A, k2);
          for (int a = 0; a < SA; ++a) k3[a] = hg * (f2[a] + rh * (c31 * k1[a] + c32 * k2[a]));
          G::solve(A, k3);
          for (int a = 0; a < SA; ++a) {
            const int i = G::ACT[a];
            yn[a] = y[i] + k1[a] + m2 * k2[a] + m3 * k3[a];
            const double e = (e1 * k1[a] + e2 * k2[a] + e3 * k3[a]) / (sc[i] + rtol * std::fmax(std::fabs(y[i]), std::fabs(yn[a])));
            err += e * e;
          }
          err = std::sqrt(err / S);
          if (!(err == err)) ok = false;
        }
        if (ok && err <= 1.0) {
          for (int a = 0; a < SA; ++a) y[G::ACT[a]] = yn[a];
          t += h;
          ++steps;
          const double fac = err > 0.0 ? 0.9 * std::pow(err, -1.0 / 3.0) : 5.0;
          h = h * std::fmin(5.0, std::fmax(0.2, fac));
        } else {
          ++rejects;
          const double fac = ok ? 0.9 * std::pow(err, -1.0 / 3.0) : 0.25;
          h = h * std::fmin(0.5, std::fmax(0.1, fac));
        }
      }
      if (steps >= 0) hnext = h;
    }
    double q = 0.0;
    for (int i = 0; i < S; ++i) {
      const double Yn = y[i] * G::W[i] / rho;
      const double rr = T >= Tmin ? (Yn - Y0[i]) * rho_rr[c] / dt : 0.0;
      RR[(long)i * n + c] = rr;
      q -= hc[i] * rr;
    }
    Qdot[c] = q;
    stats[c] = steps;
    stats[n + c] = rejects;
    if (hnext > 0.0) stats[2 * n + c] = hnext;
    if (steps < 0) ++fail;
  }
  return fail;
}

void chem_solve(Ctx& x, double dt, const char* rho_field) {
  CHECK(x.R > 0, "chemistry mechanism not set (dfmi_chem_set_mechanism)");
  CHECK(x.generated != 0, "CPU-A integrates the compiled-in mechanisms only (burke9, es80)");
  const double* rho_rr = x.f(rho_field);
  const int nf = x.generated == 1 ? chem_cells<ChemGen_burke9>(x, dt, rho_rr) : chem_cells<ChemGen_es80>(x, dt, rho_rr);
  CHECK(nf == 0, "chemistry: " + std::to_string(nf) + " cell(s) hit the integrator step limit (max_steps = " +
                     std::to_string(x.max_steps) + ")");
}

// ---------------------------------------------------------------- equations (oracle.py time_step order)
void copy(Ctx& x, const char* dst, const char* src) {
  std::vector<double>& d = x.fields.at(dst).v;
  const std::vector<double>& s = x.fields.at(src).v;
#pragma omp parallel for schedule(static)
  for (size_t i = 0; i < d.size(); ++i) d[i] = s[i];
}

void pre_time_step(Ctx& x) {   // dfMatrixDataBase::preTimeStep
  for (auto pr : {std::make_pair("rho_old", "rho"), std::make_pair("boundary_rho_old", "boundary_rho"),
                  std::make_pair("phi_old", "phi"), std::make_pair("boundary_phi_old", "boundary_phi"),
                  std::make_pair("U_old", "U"), std::make_pair("boundary_U_old", "boundary_U"),
                  std::make_pair("K_old", "K"), std::make_pair("p_old", "p"), std::make_pair("boundary_p_old", "boundary_p")})
    copy(x, pr.first, pr.second);
}

void kinetic(Ctx& x) {
  const double *U = x.f("U"), *bU = x.f("boundary_U");
  double *K = x.f("K"), *bK = x.f("boundary_K");
  const long C = x.C, B = x.B;
#pragma omp parallel for schedule(static)
  for (long c = 0; c < C; ++c) K[c] = 0.5 * (U[c] * U[c] + U[C + c] * U[C + c] + U[2 * C + c] * U[2 * C + c]);
  for (long b = 0; b < B; ++b) bK[b] = 0.5 * (bU[b] * bU[b] + bU[B + b] * bU[B + b] + bU[2 * B + b] * bU[2 * B + b]);
}

void do_U(Ctx& x) {
  orc(orc_u_assemble(), "UEqn");
  const long C = x.C, F = x.F, B = x.B;
  for (auto k : {"lower", "upper"}) std::memcpy(x.w(std::string("ueqn_") + k), x.w(std::string("out_") + k), F * sizeof(double));
  std::memcpy(x.w("ueqn_source"), x.w("out_source"), 3 * C * sizeof(double));
  std::memcpy(x.w("ueqn_internal_coeffs"), x.w("out_internal_coeffs"), 3 * B * sizeof(double));
  std::memcpy(x.w("ueqn_boundary_coeffs"), x.w("out_boundary_coeffs"), 3 * B * sizeof(double));
  double* U = x.f("U");
  for (int k = 0; k < 3; ++k)
    solve(x, "U", x.w("out_lower"), x.w("out_upper"), x.w("out_diag"), x.w("out_source_solve") + k * C,
          x.w("out_internal_coeffs") + k * B, x.w("out_boundary_coeffs") + k * B, "U", U + k * C, k == 0);
  orc(orc_correct_bc("U", "boundary_U", "ptype_U", 3), "U boundary");
  kinetic(x);
}

void do_Y(Ctx& x) {
  if (x.mode == 1) chem_solve(x, 1.0 / x.rdt, "rho_old");   // thermo density of the step start (chem.hip)
  CHECK(x.mode != 2, "DNN chemistry is a GPU-path feature");
  orc(orc_conv_weights(), "div(phi,Yi_h) weights");
  orc(orc_y_prep(), "YEqn prep");
  if (study("no_diffAlphaD")) {
    std::fill_n(x.f("diffAlphaD"), x.C, 0.0);
    std::fill_n(x.f("boundary_diffAlphaD"), x.B, 0.0);
  }
  if (study("no_hDiffCorrFlux")) {
    std::fill_n(x.f("hDiffCorrFlux"), 3 * x.C, 0.0);
    std::fill_n(x.f("boundary_hDiffCorrFlux"), 3 * x.B, 0.0);
  }
  scale_field(x, "diffAlphaD", x.C, study_scale("dAD"));
  scale_field(x, "boundary_diffAlphaD", x.B, study_scale("dAD"));
  scale_field(x, "hDiffCorrFlux", 3 * x.C, study_scale("hdcf"));
  scale_field(x, "boundary_hDiffCorrFlux", 3 * x.B, study_scale("hdcf"));
  orc(orc_y_assemble(), "YEqn");
  const long C = x.C, F = x.F, B = x.B;
  double* Y = x.f("Y");
  bool first = true;
  for (int s = 0; s < x.S; ++s) {
    if (s == x.inert) continue;
    solve(x, "Y", x.w("out_lower") + s * F, x.w("out_upper") + s * F, x.w("out_diag") + s * C, x.w("out_source") + s * C,
          x.w("out_internal_coeffs") + s * B, x.w("out_boundary_coeffs") + s * B, "Y", Y + s * C, first);
    first = false;
  }
  orc(orc_y_inert(), "Y inert");
}

void do_E(Ctx& x) {
  orc(orc_energy_gradient(), "energy gradient");
  orc(orc_correct_bc("he", "boundary_he", "ptype_he", 1), "he boundary");
  if (study("no_dpdt")) std::fill_n(x.f("dpdt"), x.C, 0.0);
  const double sd = study_scale("dpdt");   // scaled for this EEqn only (pEqn rewrites dpdt from p)
  std::vector<double> keep;
  if (sd != 1.0) { keep.assign(x.f("dpdt"), x.f("dpdt") + x.C); scale_field(x, "dpdt", x.C, sd); }
  orc(orc_e_assemble(), "EEqn");
  if (sd != 1.0) std::copy(keep.begin(), keep.end(), x.f("dpdt"));
  solve(x, "E", x.w("out_lower"), x.w("out_upper"), x.w("out_diag"), x.w("out_source"), x.w("out_internal_coeffs"),
        x.w("out_boundary_coeffs"), "he", x.f("he"), true);
  orc(orc_correct_bc("he", "boundary_he", "ptype_he", 1), "he boundary");
}

void rho_from_psi(Ctx& x) {   // dfThermo::updateRho
  for (auto pre : {"", "boundary_"}) {
    const std::string P(pre);
    double *r = x.f(P + "rho"), *p = x.f(P + "p"), *psi = x.f(P + "psi");
    const long n = x.fields.at(P + "rho").n;
#pragma omp parallel for schedule(static)
    for (long i = 0; i < n; ++i) r[i] = p[i] * psi[i];
  }
}
void psip0(Ctx& x) {
  for (auto pre : {"", "boundary_"}) {
    const std::string P(pre);
    double *o = x.f(P + "psip0"), *p = x.f(P + "p"), *psi = x.f(P + "psi");
    const long n = x.fields.at(P + "rho").n;
#pragma omp parallel for schedule(static)
    for (long i = 0; i < n; ++i) o[i] = psi[i] * p[i];
  }
}
void correct_psip_rho(Ctx& x) {
  for (auto pre : {"", "boundary_"}) {
    const std::string P(pre);
    double *r = x.f(P + "rho"), *o = x.f(P + "psip0"), *p = x.f(P + "p"), *psi = x.f(P + "psi");
    const long n = x.fields.at(P + "rho").n;
#pragma omp parallel for schedule(static)
    for (long i = 0; i < n; ++i) r[i] = r[i] + (psi[i] * p[i] - o[i]);
  }
}

void do_p(Ctx& x) {
  orc(orc_p_assemble(), "pEqn");
  const long F = x.F, B = x.B;
  for (auto k : {"lower", "upper", "phiHbyA"}) std::memcpy(x.w(std::string("peqn_") + k), x.w(std::string("out_") + k), F * sizeof(double));
  for (auto k : {"internal_coeffs", "boundary_coeffs", "boundary_phiHbyA"})
    std::memcpy(x.w(std::string("peqn_") + k), x.w(std::string("out_") + k), B * sizeof(double));
  std::memcpy(x.f("rhorAUf"), x.w("out_rhorAUf"), F * sizeof(double));
  std::memcpy(x.f("phiHbyA"), x.w("out_phiHbyA"), F * sizeof(double));
  solve(x, "p", x.w("out_lower"), x.w("out_upper"), x.w("out_diag"), x.w("out_source"), x.w("out_internal_coeffs"),
        x.w("out_boundary_coeffs"), "p", x.f("p"), true);
  orc(orc_p_post(), "pEqn post");
}

void time_step(Ctx& x, int n_corr) {
  pre_time_step(x);
  orc(orc_rho_eqn(), "rhoEqn");
  do_U(x);
  do_Y(x);
  do_E(x);
  orc(orc_thermo_correct(0), "correctThermo");
  for (int i = 0; i < n_corr; ++i) {
    rho_from_psi(x);
    psip0(x);
    orc(orc_u_hbya(), "HbyA");
    do_p(x);
    correct_psip_rho(x);
    orc(orc_rho_eqn(), "rhoEqn");
  }
  rho_from_psi(x);
}

void copy_field(Ctx& x, const std::string& name, double* host, long count, int layout, bool to_ctx) {
  auto it = x.fields.find(name);
  CHECK(it != x.fields.end(), "unknown field '" + name + "'");
  Field& f = it->second;
  CHECK(count == f.n, "field '" + name + "': expected " + std::to_string(f.n) + " values per component, got " +
                          std::to_string(count));
  const bool aos = layout == DFMI_AOS && (f.ncomp == 3 || f.ncomp == 9);
  for (long i = 0; i < f.n; ++i)
    for (int k = 0; k < f.ncomp; ++k) {
      double& d = f.v[(size_t)k * f.n + i];
      double& h = host[aos ? i * f.ncomp + k : (long)k * f.n + i];
      if (to_ctx) d = h; else h = d;
    }
}

}  // namespace

struct dfmi_ctx { Ctx x; };

extern "C" {

const char* dfmi_version(void) {
  static std::string v;
  v = "dfmi CPU-A (OpenMP, " + std::to_string(omp_get_max_threads()) + " threads)";
  return v.c_str();
}
int dfmi_last_error(char* buf, int len) {
  if (buf && len > 0) std::snprintf(buf, len, "%s", g_err.c_str());
  return (int)g_err.size();
}
int dfmi_create(dfmi_ctx** out, int) { return guard([&] { CHECK(out, "null output pointer"); *out = new dfmi_ctx(); }); }
int dfmi_destroy(dfmi_ctx* ctx) { delete ctx; return 0; }

int dfmi_set_constant_values(dfmi_ctx* ctx, int num_cells, int num_total_cells, int num_surfaces, int num_boundary_surfaces,
                             int num_patches, int num_proc_surfaces, const int* patch_size, int num_species, double rdelta_t) {
  return guard([&] {
    Ctx& x = ctx->x;
    CHECK(num_cells > 0 && num_surfaces >= 0 && num_boundary_surfaces >= 0 && num_patches >= 0, "bad sizes");
    CHECK(num_proc_surfaces == 0, "CPU-A runs one rank (no processor patches)");
    CHECK(num_species >= 2 && num_species <= 64, "num_species must be in [2,64]");
    CHECK(rdelta_t > 0, "rdelta_t must be positive");
    x.C = num_cells; x.Ctot = num_total_cells; x.F = num_surfaces; x.B = num_boundary_surfaces; x.P = num_patches;
    x.S = num_species; x.rdt = rdelta_t;
    x.psize.assign(patch_size, patch_size + num_patches);
    x.pkind.assign(num_patches, 0);
    x.cyc_nbr.assign(num_patches, -1);
    x.have_sizes = true;
  });
}
int dfmi_set_cyclic_info(dfmi_ctx* ctx, const int* cyc) {
  return guard([&] { CHECK(ctx->x.have_sizes, "call dfmi_set_constant_values first"); ctx->x.cyc_nbr.assign(cyc, cyc + ctx->x.P); });
}
int dfmi_set_comm_info(dfmi_ctx*, const void*, int, int, const int*) {
  return guard([&] { throw Error("dfmi (CPU-A): single rank only"); });
}
int dfmi_get_unique_id(void*) { return guard([&] { throw Error("dfmi (CPU-A): no RCCL"); }); }
int dfmi_set_comm_local(dfmi_ctx*, int, int, int, const int*) { return guard([&] { throw Error("dfmi (CPU-A): single rank only"); }); }

int dfmi_set_constant_indexes(dfmi_ctx* ctx, const int* owner, const int* neighbour, const int*, const int*, int) {
  return guard([&] {
    Ctx& x = ctx->x;
    CHECK(x.have_sizes, "call dfmi_set_constant_values first");
    for (int f = 0; f < x.F; ++f) {
      CHECK(owner[f] >= 0 && neighbour[f] < x.C && owner[f] < neighbour[f], "owner/neighbour out of range or not upper-triangular");
      CHECK(f == 0 || owner[f - 1] < owner[f] || (owner[f - 1] == owner[f] && neighbour[f - 1] < neighbour[f]),
            "faces are not in upper-triangular order");
    }
    x.own.assign(owner, owner + x.F);
    x.nei.assign(neighbour, neighbour + x.F);
    if (x.own.empty()) { x.own.push_back(0); x.nei.push_back(0); }
    x.have_topo = true;
  });
}
int dfmi_init_constant_fields_internal(dfmi_ctx* ctx, const double* sf, const double* mag_sf, const double* weight,
                                       const double* delta_coeffs, const double* volume, const double* mesh_distance) {
  return guard([&] {
    Ctx& x = ctx->x;
    CHECK(x.have_topo, "call dfmi_set_constant_indexes first");
    const long F = x.F;
    std::vector<double> s(3 * std::max(F, 1L)), md(3 * std::max(F, 1L), 0.0);
    for (long f = 0; f < F; ++f) for (int k = 0; k < 3; ++k) s[k * F + f] = sf[f * 3 + k];
    if (mesh_distance) for (long f = 0; f < F; ++f) for (int k = 0; k < 3; ++k) md[k * F + f] = mesh_distance[f * 3 + k];
    x.work["sf"] = s;
    x.work["mesh_distance"] = md;   // the limited schemes' d (LimitedScheme::calcLimiter)
    x.work["mag_sf"].assign(mag_sf, mag_sf + F);
    x.work["weight"].assign(weight, weight + F);
    x.work["delta_coeffs"].assign(delta_coeffs, delta_coeffs + F);
    x.work["volume"].assign(volume, volume + x.C);
    for (auto n : {"mag_sf", "weight", "delta_coeffs"}) if (x.work[n].empty()) x.work[n].push_back(0.0);
    x.have_geom = true;
  });
}
int dfmi_init_constant_fields_boundary(dfmi_ctx* ctx, const double* bsf, const double* bmag, const double* bdelta,
                                       const double* bweight, const int* bface_cell, const int* ptype_calc,
                                       const int* ptype_extrap) {
  return guard([&] {
    Ctx& x = ctx->x;
    CHECK(x.have_geom, "call dfmi_init_constant_fields_internal first");
    const long B = x.B;
    for (int p = 0; p < x.P; ++p) {
      const int t = ptype_calc[p];
      CHECK(t != PROC && t != PROC_CYC, "CPU-A runs one rank (no processor patches)");
      x.pkind[p] = t == CYCLIC ? 1 : 0;
    }
    x.bfc.assign(bface_cell, bface_cell + B);
    std::vector<double> s(3 * std::max(B, 1L));
    for (long b = 0; b < B; ++b) for (int k = 0; k < 3; ++k) s[k * B + b] = bsf[b * 3 + k];
    x.work["boundary_sf"] = s;
    x.work["boundary_mag_sf"].assign(bmag, bmag + B);
    x.work["boundary_delta_coeffs"].assign(bdelta, bdelta + B);
    x.work["boundary_weight"].assign(bweight, bweight + B);
    for (auto n : {"boundary_mag_sf", "boundary_delta_coeffs", "boundary_weight"}) if (x.work[n].empty()) x.work[n].push_back(0.0);
    // slot topology
    x.poff.assign(x.P + 1, 0);
    x.slot_patch.assign(B, -1);
    x.prim.assign(B, 1);
    int off = 0;
    for (int p = 0; p < x.P; ++p) { x.poff[p] = off; for (int i = 0; i < x.psize[p]; ++i) x.slot_patch[off + i] = p; off += x.psize[p]; }
    x.poff[x.P] = off;
    CHECK(off == B, "patch sizes do not add up to num_boundary_surfaces");
    x.partner.assign(B, -1);
    for (int p = 0; p < x.P; ++p) {
      if (x.pkind[p] != 1) continue;
      const int q = x.cyc_nbr[p];
      CHECK(q >= 0 && q < x.P && x.psize[q] == x.psize[p], "cyclic patch without a matching neighbour patch");
      for (int i = 0; i < x.psize[p]; ++i) x.partner[x.poff[p] + i] = x.bfc[x.poff[q] + i];
    }
    if (x.bfc.empty()) x.bfc.push_back(0);
    x.ptype["calculated"].assign(ptype_calc, ptype_calc + x.P);
    x.ptype["extrapolated"].assign(ptype_extrap, ptype_extrap + x.P);
    allocate_fields(x);
    build_rows(x);
    x.amg_ready = false;
    x.have_bgeom = true;
  });
}

int dfmi_renumber_cells(int, const double*, int, const int*, const int*, const char*, int*) {
  return guard([&] { throw Error("dfmi (CPU-A): renumbering is provided by the GPU library"); });
}
int dfmi_renumber_faces(int, int, const int*, const int*, const int*, int*, int*, int*, int*) {
  return guard([&] { throw Error("dfmi (CPU-A): renumbering is provided by the GPU library"); });
}

int dfmi_set_traversal(dfmi_ctx*, const int*) { return 0; }   // a GPU visiting order: nothing to do here

int dfmi_init_boundary_delta(dfmi_ctx* ctx, const double* bd) {
  return guard([&] {
    Ctx& x = ctx->x;
    CHECK(x.have_bgeom, "call dfmi_init_constant_fields_boundary first");
    std::vector<double> s(3 * std::max(x.B, 1), 0.0);
    for (long b = 0; b < x.B; ++b) for (int k = 0; k < 3; ++k) s[k * x.B + b] = bd[b * 3 + k];
    x.work["boundary_delta"] = s;
  });
}

// the same selection as the HIP library (include/dfmi.h dfmi_set_scheme); the arithmetic is the oracle's
int dfmi_set_scheme(dfmi_ctx* ctx, const char* term, const char* scheme) {
  return guard([&] {
    Ctx& x = ctx->x;
    const std::string t(term ? term : "");
    std::vector<std::string> tok;
    std::string cur;
    for (char ch : std::string(scheme ? scheme : "") + " ") {
      if (ch == ' ' || ch == '\t') { if (!cur.empty()) tok.push_back(cur); cur.clear(); } else cur += ch;
    }
    if (!tok.empty() && tok[0] == "Gauss") tok.erase(tok.begin());
    CHECK(!tok.empty(), t + ": empty scheme");
    int kind = -1;
    double k = 1.0;
    if (tok[0] == "upwind") kind = 0;
    else if (tok[0] == "linear") kind = 1;
    else if (tok[0] == "limitedLinear") kind = 2;
    else if (tok[0] == "limitedLinear01") kind = 3;
    else if (tok[0] == "cubic") kind = 4;
    else if (tok[0] == "limitedLinearV") kind = 5;
    CHECK(kind >= 0, t + ": unsupported scheme");
    if (kind == 2 || kind == 3 || kind == 5) {
      CHECK(tok.size() == 2, t + ": limitedLinear needs its coefficient k");
      k = std::stod(tok[1]);
      CHECK(k >= 0 && k <= 1, t + ": limitedLinear coefficient must be in [0, 1]");
    } else CHECK(tok.size() == 1, t + ": unexpected arguments");
    if (t == "div(phi,Yi_h)") { CHECK(kind == 0 || kind == 2 || kind == 3, t + ": upwind or limitedLinear(01)"); x.schemes[0] = kind; x.scheme_k[0] = k; }
    else if (t == "div(phi,K)") { CHECK(kind <= 3, t + ": upwind, linear or limitedLinear(01)"); x.schemes[1] = kind; x.scheme_k[1] = k; }
    else if (t == "div(hDiffCorrFlux)") { CHECK(kind == 1 || kind == 4, t + ": linear or cubic"); x.schemes[2] = kind; }
    else if (t == "div(phi,U)") { CHECK(kind == 1 || kind == 5, t + ": linear or limitedLinearV"); x.schemes[3] = kind; x.scheme_k[2] = k; }
    else throw Error("dfmi (CPU-A): unknown scheme term '" + t + "'");
  });
}

int dfmi_set_patch_types(dfmi_ctx* ctx, const char* field, const int* pt) {
  return guard([&] {
    Ctx& x = ctx->x;
    CHECK(x.have_bgeom, "call dfmi_init_constant_fields_boundary first");
    const std::string f(field);
    CHECK(f == "U" || f == "p" || f == "he" || f == "K" || f == "Y" || f == "T" || f == "rho", "unknown patch-type field '" + f + "'");
    for (int p = 0; p < x.P; ++p) {
      CHECK(pt[p] >= 0 && pt[p] <= 12 && pt[p] != COUPLED, "unsupported boundary condition code");
      CHECK((x.pkind[p] == 1) == (pt[p] == CYCLIC), "field type disagrees with the mesh patch kind");
      CHECK(pt[p] != WAVE || f == "p", "waveTransmissive is supported for p");
    }
    x.ptype[f].assign(pt, pt + x.P);
  });
}
int dfmi_set_patch_param(dfmi_ctx* ctx, const char* field, int patch, const char* name, double value) {
  return guard([&] {
    Ctx& x = ctx->x;
    CHECK(x.have_bgeom && patch >= 0 && patch < x.P, "bad patch");
    CHECK(std::string(field) == "p" && std::string(name) == "gamma", "patch parameters: ('p', 'gamma')");
    double* g = x.f("boundary_p_gamma");
    for (int i = 0; i < x.psize[patch]; ++i) g[x.poff[patch] + i] = value;
  });
}
int dfmi_set_inert_index(dfmi_ctx* ctx, int i) {
  return guard([&] { CHECK(i >= 0 && i < ctx->x.S, "inert index out of range"); ctx->x.inert = i; });
}
int dfmi_thermo_set_coeffs(dfmi_ctx* ctx, int S, const double* W, const double* nasa, const double* visc, const double* cond,
                           const double* bdiff) {
  return guard([&] {
    Ctx& x = ctx->x;
    CHECK(x.have_sizes && S == x.S, "thermo species count differs from num_species");
    x.W.assign(W, W + S); x.nasa.assign(nasa, nasa + 15 * S); x.visc.assign(visc, visc + 5 * S);
    x.cond.assign(cond, cond + 5 * S); x.bdiff.assign(bdiff, bdiff + 5 * S * S);
  });
}
int dfmi_thermo_load(dfmi_ctx*, const char*) { return guard([&] { throw Error("dfmi (CPU-A): use dfmi_thermo_set_coeffs"); }); }

int dfmi_set_field(dfmi_ctx* ctx, const char* name, const double* host, long count, int layout) {
  return guard([&] { copy_field(ctx->x, name, const_cast<double*>(host), count, layout, true); });
}
int dfmi_get_field(dfmi_ctx* ctx, const char* name, double* host, long count, int layout) {
  return guard([&] { copy_field(ctx->x, name, host, count, layout, false); });
}

int dfmi_pre_time_step(dfmi_ctx* ctx) { return guard([&] { require_ready(ctx->x); pre_time_step(ctx->x); }); }
int dfmi_post_time_step(dfmi_ctx* ctx) { return guard([&] { require_ready(ctx->x); }); }
int dfmi_rho_process(dfmi_ctx* ctx) { return guard([&] { require_ready(ctx->x); orc(orc_rho_eqn(), "rhoEqn"); }); }
int dfmi_U_process(dfmi_ctx* ctx) { return guard([&] { require_ready(ctx->x); do_U(ctx->x); }); }
int dfmi_Y_process(dfmi_ctx* ctx) { return guard([&] { require_ready(ctx->x); do_Y(ctx->x); }); }
int dfmi_E_process(dfmi_ctx* ctx) { return guard([&] { require_ready(ctx->x); do_E(ctx->x); }); }
int dfmi_p_process(dfmi_ctx* ctx) { return guard([&] { require_ready(ctx->x); do_p(ctx->x); }); }
int dfmi_U_get_HbyA(dfmi_ctx* ctx) { return guard([&] { require_ready(ctx->x); orc(orc_u_hbya(), "HbyA"); }); }
int dfmi_thermo_correct(dfmi_ctx* ctx) { return guard([&] { require_ready(ctx->x); orc(orc_thermo_correct(0), "thermo"); }); }
int dfmi_thermo_update_energy(dfmi_ctx* ctx) { return guard([&] { require_ready(ctx->x); orc(orc_thermo_correct(1), "thermo"); }); }
int dfmi_thermo_update_rho(dfmi_ctx* ctx) { return guard([&] { require_ready(ctx->x); rho_from_psi(ctx->x); }); }
int dfmi_thermo_psip0(dfmi_ctx* ctx) { return guard([&] { require_ready(ctx->x); psip0(ctx->x); }); }
int dfmi_thermo_correct_psip_rho(dfmi_ctx* ctx) { return guard([&] { require_ready(ctx->x); correct_psip_rho(ctx->x); }); }
int dfmi_time_step(dfmi_ctx* ctx, int n_corr) { return guard([&] { require_ready(ctx->x); time_step(ctx->x, n_corr); }); }
int dfmi_sync(dfmi_ctx*) { return 0; }
// no device events on the CPU: the bench times CPU-A with host clocks
int dfmi_step_timer(dfmi_ctx*, int) { return 0; }
// CPU-A runs one fixed configuration (the GPU path's defaults: AMG omega 0.9, over-correction 1.4, 6 coarsest sweeps, ...)
int dfmi_set_option(dfmi_ctx*, const char* key, double) {
  return guard([&] { throw Error(std::string("dfmi (CPU-A): option '") + key + "' is not configurable here"); });
}
int dfmi_get_option(dfmi_ctx*, const char* key, double*) {
  return guard([&] { throw Error(std::string("dfmi (CPU-A): option '") + key + "' is not configurable here"); });
}
int dfmi_step_times(dfmi_ctx*, double*, int, int* got) { if (got) *got = 0; return 0; }
int dfmi_hbm_copy_peak(dfmi_ctx*, double, int, double*) { return guard([&] { throw Error("dfmi (CPU-A): no device memory"); }); }

int dfmi_correct_boundary(dfmi_ctx* ctx, const char* field) {
  return guard([&] {
    Ctx& x = ctx->x;
    require_ready(x);
    const std::string f(field);
    const int nc = f == "U" ? 3 : (f == "Y" ? x.S : 1);
    CHECK(f == "U" || f == "Y" || f == "p" || f == "he" || f == "T" || f == "rho" || f == "K", "unsupported field '" + f + "'");
    orc(orc_correct_bc(f.c_str(), ("boundary_" + f).c_str(), ("ptype_" + f).c_str(), nc), "correct_boundary");
  });
}

int dfmi_assemble(dfmi_ctx*, const char*) { return guard([&] { throw Error("dfmi (CPU-A): matrix inspection is a GPU-path feature"); }); }
int dfmi_get_matrix(dfmi_ctx*, const char*, const char*, double*, long) { return guard([&] { throw Error("dfmi (CPU-A): matrix inspection is a GPU-path feature"); }); }
int dfmi_get_solver_rows(dfmi_ctx*, const char*, const char*, double*, long) { return guard([&] { throw Error("dfmi (CPU-A): matrix inspection is a GPU-path feature"); }); }

int dfmi_set_solver(dfmi_ctx* ctx, const char* eqn, int max_iter, double tol, double abs_tol) {
  return guard([&] {
    const std::string e(eqn);
    CHECK(e == "U" || e == "Y" || e == "E" || e == "p", "unknown equation '" + e + "'");
    CHECK(max_iter > 0 && tol >= 0 && abs_tol >= 0, "bad solver controls");
    SolverCfg& c = ctx->x.solver[e];
    if (!ctx->x.solver.count(e) || c.max_iter == 0) c.precond = e == "p" ? 1 : 0;
    c.max_iter = max_iter; c.tol = tol; c.abs_tol = abs_tol;
  });
}
int dfmi_set_preconditioner(dfmi_ctx* ctx, const char* eqn, const char* name) {
  return guard([&] {
    const std::string e(eqn), n(name);
    CHECK(n == "jacobi" || (n == "amg" && e == "p"), "preconditioner: 'jacobi', or 'amg' for p");
    ctx->x.solver[e].precond = n == "amg" ? 1 : 0;
  });
}
int dfmi_amg_info(dfmi_ctx* ctx, int max_levels, int* n_levels, int* cells, int* width) {
  return guard([&] {
    Ctx& x = ctx->x;
    if (n_levels) *n_levels = (int)x.amg.size();
    for (int l = 0; l < (int)x.amg.size() && l < max_levels; ++l) { cells[l] = x.amg[l].n; width[l] = x.amg[l].W; }
  });
}
int dfmi_row_classes(dfmi_ctx*, int* n) {   // explicit CSR rows on the CPU
  if (n) *n = 0;
  return 0;
}
int dfmi_hex_dims(dfmi_ctx*, int* nx, int* ny, int* nz) {
  if (nx) *nx = 0;
  if (ny) *ny = 0;
  if (nz) *nz = 0;
  return 0;
}
int dfmi_solver_stats(dfmi_ctx* ctx, const char* eqn, int* iters, double* res0, double* rel) {
  return guard([&] {
    auto it = ctx->x.stats.find(eqn);
    CHECK(it != ctx->x.stats.end(), std::string("no solve recorded for ") + eqn);
    if (iters) *iters = it->second.iters;
    if (res0) *res0 = it->second.res0;
    if (rel) *rel = it->second.res;
  });
}
int dfmi_solver_work(dfmi_ctx* ctx, const char* eqn, double* iters, int reset) {
  return guard([&] {
    Stats& s = ctx->x.stats[eqn];
    if (iters) *iters = s.work;
    if (reset) s.work = 0;
  });
}

int dfmi_chem_set_mechanism(dfmi_ctx* ctx, int R, const int* idata, const int* irs, const double* dd) {
  return guard([&] {
    Ctx& x = ctx->x;
    CHECK(x.have_sizes && R > 0, "bad mechanism");
    CHECK(!x.W.empty(), "set the thermo coefficients before the mechanism");
    x.R = R;
    x.idata.assign(idata, idata + (size_t)R * 8);
    x.irs.assign(irs, irs + (size_t)R * 6);
    x.dd.assign(dd, dd + (size_t)R * (17 + x.S));
    unsigned long long fp = 0xcbf29ce484222325ull;   // the fingerprint chem.hip matches (chem_codegen.fingerprint)
    const int S32 = x.S;
    fp = fnv(fp, &S32, 4);
    fp = fnv(fp, x.idata.data(), x.idata.size() * 4);
    fp = fnv(fp, x.irs.data(), x.irs.size() * 4);
    fp = fnv(fp, x.dd.data(), x.dd.size() * 8);
    fp = fnv(fp, x.nasa.data(), x.nasa.size() * 8);
    fp = fnv(fp, x.W.data(), x.W.size() * 8);
    x.generated = fp == ChemGen_burke9::FINGERPRINT ? 1 : (fp == ChemGen_es80::FINGERPRINT ? 2 : 0);
  });
}
int dfmi_chem_set_options(dfmi_ctx* ctx, int mode, double rtol, double atol, double T_min) {
  return guard([&] {
    CHECK(mode >= 0 && mode <= 1, "CPU-A chemistry mode: 0 (off) or 1 (ODE)");
    CHECK(rtol > 0 && atol > 0, "chemistry tolerances must be positive");
    Ctx& x = ctx->x;
    x.mode = mode; x.rtol = rtol; x.atol = atol; x.Tmin = T_min;
  });
}
int dfmi_chem_solve(dfmi_ctx* ctx, double dt) {
  return guard([&] { require_ready(ctx->x); CHECK(dt > 0, "dt must be positive"); chem_solve(ctx->x, dt, "rho"); });
}
int dfmi_chem_set_max_steps(dfmi_ctx* ctx, int n) { return guard([&] { CHECK(n > 0, "max_steps must be positive"); ctx->x.max_steps = n; }); }
int dfmi_chem_info(dfmi_ctx* ctx, int* generated) { return guard([&] { if (generated) *generated = ctx->x.generated; }); }
// df0DFoam steps (df0DFoam.C:99-113; the GPU path's zero_d_step, fv_kernels.hip): chemistry at the
// current density, YEqn ddt(rho, Y) == RR with clipping and the inert remainder, he held, correctThermo
int dfmi_zero_d_step(dfmi_ctx* ctx, double dt, int n_steps) {
  return guard([&] {
    Ctx& x = ctx->x;
    require_ready(x);
    CHECK(dt > 0 && n_steps >= 1, "0D step: dt and n_steps must be positive");
    CHECK(x.mode == 1, "CPU-A 0D step: chemistry mode must be 1 (ODE)");
    const long C = x.C;
    const int S = x.S, inert = x.inert;
    for (int it = 0; it < n_steps; ++it) {
      std::memcpy(x.f("rho_old"), x.f("rho"), C * sizeof(double));
      chem_solve(x, dt, "rho");
      const double rdt = 1.0 / dt;
      const double *V = x.w("volume"), *ro = x.f("rho_old"), *rho = x.f("rho"), *RR = x.f("RR");
      double* Y = x.f("Y");
#pragma omp parallel for schedule(static)
      for (long c = 0; c < C; ++c) {
        const double vol = V[c], dg = rdt * rho[c] * vol, r0 = rdt * ro[c];
        double sum = 0.0;
        for (int s = 0; s < S; ++s) {
          if (s == inert) continue;
          double y = (r0 * Y[s * C + c] * vol + vol * RR[s * C + c]) / dg;
          y = y > 0 ? y : 0;
          Y[s * C + c] = y;
          sum += y;
        }
        sum = 1 - sum;
        Y[inert * C + c] = sum > 0 ? sum : 0;
      }
      orc(orc_correct_bc("Y", "boundary_Y", "ptype_Y", S), "Y boundary");
      orc(orc_thermo_correct(0), "correctThermo");
      rho_from_psi(x);
    }
  });
}

int dfmi_dnn_set_model(dfmi_ctx*, int, int, const int*, const float*, const double*, const double*, const double*,
                       const double*, double, double) {
  return guard([&] { throw Error("dfmi (CPU-A): DNN chemistry is a GPU-path feature"); });
}
int dfmi_dnn_load_model(dfmi_ctx*, const char*, double, double) {
  return guard([&] { throw Error("dfmi (CPU-A): DNN chemistry is a GPU-path feature"); });
}
int dfmi_dnn_infer(dfmi_ctx*, int*) { return guard([&] { throw Error("dfmi (CPU-A): DNN chemistry is a GPU-path feature"); }); }
int dfmi_dnn_stats(dfmi_ctx*, int*, double*) { return guard([&] { throw Error("dfmi (CPU-A): DNN chemistry is a GPU-path feature"); }); }
int dfmi_kernel_timer(dfmi_ctx*, const char*) { return guard([&] { throw Error("dfmi (CPU-A): no kernels"); }); }
int dfmi_kernel_time(dfmi_ctx*, double*, int*) { return guard([&] { throw Error("dfmi (CPU-A): no kernels"); }); }
int dfmi_kernel_time_named(dfmi_ctx*, const char*, double*, int*) { return guard([&] { throw Error("dfmi (CPU-A): no kernels"); }); }
int dfmi_comm_timer(dfmi_ctx*, int) { return guard([&] { throw Error("dfmi (CPU-A): one rank, no communication"); }); }
int dfmi_comm_report(dfmi_ctx*, char*, int, int*) { return guard([&] { throw Error("dfmi (CPU-A): one rank, no communication"); }); }

}  // extern "C"
