// capi.cpp -- extern "C" boundary (include/dfmi.h) and the PIMPLE orchestration.
//
// Host side of the drop-in: what createGPUSolver.H + dfLowMachFoam.C do with the reference's
// C++ classes (dfMatrixDataBase, dfRhoEqn, dfUEqn, dfYEqn, dfEEqn, dfpEqn, dfThermo) is exposed
// here as plain C entry points with pointers and sizes. All device work is stream-ordered on one
// HIP stream per context; the host synchronises only where the reference reads back to the host
// (solver residual checks, dfmi_get_field, dfmi_sync).
#include "dfmi_ctx.h"
#include "../../include/dfmi.h"
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <numeric>

struct dfmi_ctx { dfmi::Ctx x; };

namespace {
thread_local std::string g_err;

template <class FN> int guard(FN&& fn) {
  try { fn(); return 0; }
  catch (std::exception& e) { g_err = e.what(); return 1; }
  catch (...) { g_err = "unknown error"; return 2; }
}

using namespace dfmi;

void alloc_field(Ctx& x, const std::string& name, long n, int ncomp, bool boundary, bool face = false) {
  Field& f = x.fields[name];
  f.n = n; f.ncomp = ncomp; f.boundary = boundary; f.face = face;
  f.buf.alloc((size_t)n * ncomp);
  f.buf.zero(x.stream);
}

void allocate_fields(Ctx& x) {
  const long C = x.C, B = x.B;
  const int S = x.S;
  for (auto n : {"rho", "rho_old", "p", "p_old", "he", "T", "K", "K_old", "psi", "mu", "alpha", "dpdt", "rAU",
                 "diffAlphaD", "psip0"}) {
    alloc_field(x, n, C, 1, false);
    alloc_field(x, std::string("boundary_") + n, B, 1, true);
  }
  for (auto n : {"U", "U_old", "HbyA", "hDiffCorrFlux", "sumYDiffError"}) {
    alloc_field(x, n, C, 3, false);
    alloc_field(x, std::string("boundary_") + n, B, 3, true);
  }
  alloc_field(x, "tauU", C, 9, false);
  alloc_field(x, "chem_stats", C, 3, false);   // per cell: accepted / rejected integrator steps, next step size
  alloc_field(x, "Qdot", C, 1, false);         // heat release -sum_i hc_i RR_i [W/m^3] (dfChemistryModel.C:771)
  alloc_field(x, "boundary_tauU", B, 9, true);
  alloc_field(x, "boundary_heGradient", B, 1, true);   // gradientEnergy patches (dfEEqn.cu:266-287)
  // mixed conditions: p's waveTransmissive valueFraction (set at each pEqn assembly) and gamma; the
  // inletValue of every field that may use inletOutlet
  alloc_field(x, "boundary_p_vf", B, 1, true);
  alloc_field(x, "boundary_p_gamma", B, 1, true);
  alloc_field(x, "boundary_U_ref", B, 3, true);
  alloc_field(x, "boundary_p_ref", B, 1, true);
  alloc_field(x, "boundary_Y_ref", B, S, true);
  alloc_field(x, "boundary_K_ref", B, 1, true);
  for (auto n : {"Y", "rhoD", "hai", "RR"}) {
    alloc_field(x, n, C, S, false);
    alloc_field(x, std::string("boundary_") + n, B, S, true);
  }
  for (auto n : {"phi", "phi_old", "phiUc", "rhorAUf", "phiHbyA"}) {
    alloc_field(x, n, x.Fs, 1, false, true);
    alloc_field(x, std::string("boundary_") + n, B, 1, true);
  }
  const long Fs = x.Fs;
  auto mk = [&](Matrix& A, int ns, int nsrc, int nb) {
    A.nsys = ns;
    A.lower.alloc((size_t)ns * Fs); A.upper.alloc((size_t)ns * Fs); A.diag.alloc((size_t)ns * C);
    A.source.alloc((size_t)nsrc * C); A.ic.alloc((size_t)nb * B); A.bc.alloc((size_t)nb * B);
    A.lower.zero(x.stream); A.upper.zero(x.stream); A.diag.zero(x.stream); A.source.zero(x.stream);
    A.ic.zero(x.stream); A.bc.zero(x.stream);
  };
  mk(x.mU, 1, 3, 3);
  x.mU.source_solve.alloc(3 * C);
  mk(x.mY, S, S, S);
  mk(x.mE, 1, 1, 1);
  mk(x.mP, 1, 1, 1);
  for (auto e : {"U", "Y", "E"}) if (!x.solver.count(e)) x.solver[e] = SolverCfg{20, 1e-5, 0.0};   // amgxUOptions
  if (!x.solver.count("p")) x.solver["p"] = SolverCfg{1000, 1e-5, 0.0, 1};   // amgxpOptions: AMG-preconditioned
}

// Build the deterministic gather topology from owner/neighbour and the boundary face cells.
void build_boundary_topology(Ctx& x) {
  const int C = x.C, B = x.B;
  x.poff.assign(x.P + 1, 0);
  std::vector<int> slot_patch(B, -1);
  std::vector<int8_t> prim(B, 0);
  int off = 0;
  for (int p = 0; p < x.P; ++p) {
    x.poff[p] = off;
    const int n = x.psize[p];
    const int slots = x.pkind[p] == 2 ? 2 * n : n;
    for (int i = 0; i < slots; ++i) { slot_patch[off + i] = p; prim[off + i] = i < n; }
    off += slots;
  }
  x.poff[x.P] = off;
  DFMI_CHECK(off == B, "patch sizes / kinds do not add up to num_boundary_surfaces");
  std::vector<int> partner(B, -1);
  for (int p = 0; p < x.P; ++p) {
    if (x.pkind[p] != 1) continue;
    const int q = x.cyc_nbr.empty() ? -1 : x.cyc_nbr[p];
    DFMI_CHECK(q >= 0 && q < x.P && x.psize[q] == x.psize[p], "cyclic patch without a matching neighbour patch");
    for (int i = 0; i < x.psize[p]; ++i) partner[x.poff[p] + i] = x.h_bfc[x.poff[q] + i];
  }
  std::vector<int> cnt(C + 1, 0);
  for (int b = 0; b < B; ++b) if (prim[b]) {
    const int c = x.h_bfc[b];
    DFMI_CHECK(c >= 0 && c < C, "boundary face cell out of range");
    cnt[c + 1]++;
  }
  for (int c = 0; c < C; ++c) cnt[c + 1] += cnt[c];
  std::vector<int> slot(cnt[C]), pos(cnt.begin(), cnt.end() - 1);
  for (int b = 0; b < B; ++b) if (prim[b]) slot[pos[x.h_bfc[b]]++] = b;
  x.cbStart.upload(cnt, x.stream);
  x.cbSlot.upload(slot.empty() ? std::vector<int>{0} : slot, x.stream);
  x.partner.upload(partner, x.stream);
  x.sprim.upload(prim.data(), prim.size(), x.stream);
  x.bfc.upload(x.h_bfc, x.stream);
}

void set_ptype(Ctx& x, const std::string& field, const int* pt) {
  std::vector<int> v(pt, pt + x.P);
  x.ptype[field] = v;
  std::vector<int8_t> s(x.B, EMPTY);
  for (int p = 0; p < x.P; ++p) {
    const int slots = x.pkind[p] == 2 ? 2 * x.psize[p] : x.psize[p];
    for (int i = 0; i < slots; ++i) s[x.poff[p] + i] = (int8_t)pt[p];
  }
  x.stype[field].upload(s.data(), s.size(), x.stream);
}

void copy_field(Ctx& x, const std::string& name, const double* host, long count, int layout, bool to_dev) {
  auto it = x.fields.find(name);
  DFMI_CHECK(it != x.fields.end(), "unknown field '" + name + "'");
  Field& f = it->second;
  if (f.face) {   // OpenFOAM face order on the host, owner-slot storage on the device
    DFMI_CHECK(count == x.F, "field '" + name + "': expected " + std::to_string(x.F) + " values, got " + std::to_string(count));
    std::vector<double> st(f.n, 0.0);
    if (to_dev) {
      for (long i = 0; i < x.F; ++i) st[x.h_fst[i]] = host[i];
      DFMI_HIP(hipMemcpyAsync(f.buf.p, st.data(), f.n * sizeof(double), hipMemcpyHostToDevice, x.stream));
      DFMI_HIP(hipStreamSynchronize(x.stream));
    } else {
      DFMI_HIP(hipMemcpyAsync(st.data(), f.buf.p, f.n * sizeof(double), hipMemcpyDeviceToHost, x.stream));
      DFMI_HIP(hipStreamSynchronize(x.stream));
      double* out = const_cast<double*>(host);
      for (long i = 0; i < x.F; ++i) out[i] = st[x.h_fst[i]];
    }
    return;
  }
  DFMI_CHECK(count == f.n, "field '" + name + "': expected " + std::to_string(f.n) + " values per component, got " +
                               std::to_string(count));
  const size_t tot = (size_t)f.n * f.ncomp;
  const bool perm = layout == DFMI_AOS && (f.ncomp == 3 || f.ncomp == 9);
  std::vector<double> tmp;
  if (to_dev) {
    const double* src = host;
    if (perm) {
      tmp.resize(tot);
      for (long i = 0; i < f.n; ++i) for (int k = 0; k < f.ncomp; ++k) tmp[(size_t)k * f.n + i] = host[i * f.ncomp + k];
      src = tmp.data();
    }
    DFMI_HIP(hipMemcpyAsync(f.buf.p, src, tot * sizeof(double), hipMemcpyHostToDevice, x.stream));
    DFMI_HIP(hipStreamSynchronize(x.stream));
  } else {
    double* dst = const_cast<double*>(host);
    if (perm) { tmp.resize(tot); dst = tmp.data(); }
    DFMI_HIP(hipMemcpyAsync(dst, f.buf.p, tot * sizeof(double), hipMemcpyDeviceToHost, x.stream));
    DFMI_HIP(hipStreamSynchronize(x.stream));
    if (perm) {
      double* out = const_cast<double*>(host);
      for (long i = 0; i < f.n; ++i) for (int k = 0; k < f.ncomp; ++k) out[i * f.ncomp + k] = tmp[(size_t)k * f.n + i];
    }
  }
}

void require_ready(Ctx& x) {
  DFMI_CHECK(x.have_sizes && x.have_topo && x.have_geom && x.have_bgeom, "mesh not fully initialised");
  if (!x.ell.ready) build_ell(x);   // gather rows (face lists of the assembly kernels, solver columns)
}

void maybe_setup_halo(Ctx& x);

// ---- equation drivers
void do_U(Ctx& x) {
  u_assemble(x);
  Matrix& A = x.mU;
  solve_bicgstab(x, "U", 3, nullptr, A.lower, 0, A.upper, 0, A.diag, 0, A.source_solve, x.C, A.ic, A.bc, x.B, "U",
                 x.f("U"), x.C, x.solver["U"]);
  u_post_solve(x);
}
// YEqn up to its assembled rows: the chemistry source, the preparation terms and the rows (no host
// synchronisation inside, so dfmi_time_step can issue it on the side stream beside the UEqn)
// weights = false: the div(phi,Yi_h) weights are formed elsewhere (do_U_Y_fork) and `rows_after` (if set) is the
// event the rows wait for on this stream
void do_Y_front(Ctx& x, bool weights = true, hipEvent_t rows_after = nullptr) {
  DFMI_CHECK(x.inert >= 0 && x.inert < x.S, "inert species index not set");
  YWs _yw(x);
  // chemistry->solve(deltaT) before YEqn (YEqn.H); the thermo density of that call is rho before this
  // step's rhoEqn, i.e. rho_old (dfChemistryModel.C:87,771; the GPU reference passes d_rho_old, dfYEqn.cu:449)
  if (x.chem.mode == 1) chem_solve(x, 1.0 / x.rdt, "rho_old");
  else if (x.chem.mode == 2) dnn_solve(x, "rho_old");   // chemistrySolver_GPU.Inference (YEqn_GPU.H)
  y_prep(x, weights);
  if (rows_after) DFMI_HIP(hipStreamWaitEvent(x.stream, rows_after, 0));
  // production path: the assembly writes the solver's ELL rows directly (no LDU round trip)
  double *val, *dS, *rhs;
  bicg_layout(x, x.S - 1, &val, &dS, &rhs);
  y_assemble_ell(x, x.ell.W, (long)x.C + x.H, val, dS, rhs);
}
void do_Y_back(Ctx& x) {
  YWs _yw(x);
  Matrix& A = x.mY;
  std::vector<int> map;
  for (int s = 0; s < x.S; ++s) if (s != x.inert) map.push_back(s);
  solve_bicgstab(x, "Y", (int)map.size(), map.data(), A.lower, x.Fs, A.upper, x.Fs, A.diag, x.C, A.source, x.C, A.ic,
                 A.bc, x.B, "Y", x.f("Y"), x.C, x.solver["Y"], true);
  y_post_solve(x);
}
void do_Y(Ctx& x) {
  do_Y_front(x);
  do_Y_back(x);
}

// The chemistry and the YEqn preparation/assembly read nothing the UEqn writes (T, p, Y, rho_old, phi, the
// thermo's transport from the last correctThermo) and the UEqn nothing they write, so they run on the side stream
// while the UEqn assembles and solves on the main one: the VALU-bound chemistry beside the memory-bound UEqn. Both
// are issued before the UEqn's convergence polls block the host. With several ranks the side stream's field halos
// (the YEqn preparation's sumYDiffError / hDiffCorrFlux, the EEqn scheme terms' gradients) go through the halo's
// second channel -- its own RCCL communicator and buffers (halo.hip) -- so the two streams' exchanges never
// interleave on one communicator; the chemistry needs no halo at all. DFMI_STEP_OVERLAP=0: off.
// While per-kernel timers are armed (dfmi_kernel_timer: the bench's roofline pass) the step runs on one
// stream, so every timed kernel has the GPU to itself and its HIP-event time is its own.
bool step_overlap(const Ctx& x) {
  static const bool on = [] { const char* e = std::getenv("DFMI_STEP_OVERLAP"); return !(e && std::atoi(e) == 0); }();
  return on && x.ktimer.targets.empty();
}
// the side stream forks from the main one and runs the YEqn front; ev_join marks its end. The side stream is the
// longer of the two (chemistry, preparation, rows against the UEqn), so the div(phi,Yi_h) weights (they read phi,
// Y, he only) run on the main stream ahead of the UEqn and the side stream waits for them just before the rows
// (the step timeline had the main stream idle for ~1 ms at the join)
void do_U_Y_fork(Ctx& x) {
  if (!x.stream2) {
    DFMI_HIP(hipStreamCreateWithFlags(&x.stream2, hipStreamNonBlocking));
    for (hipEvent_t* e : {&x.ev_fork, &x.ev_join, &x.ev_u, &x.ev_e, &x.ev_cw, &x.ev_th, &x.ev_tr})
      DFMI_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
  }
  DFMI_HIP(hipEventRecord(x.ev_fork, x.stream));
  DFMI_HIP(hipStreamWaitEvent(x.stream2, x.ev_fork, 0));
  // the weights' event is recorded on the main stream right after the weights, before the side stream's
  // hipStreamWaitEvent on it is issued (inside do_Y_front: a wait binds to the event's most recent record at call
  // time, so the record must come first); the side stream's chemistry and preparation do not wait for it
  conv_weights(x);
  // (the YEqn preparation on the main stream ahead of the UEqn instead, the side stream holding the chemistry and the
  // rows only: 14.02 / 14.05 -> 14.52 / 14.40 ms per step, round 6 -- not kept)
  DFMI_HIP(hipEventRecord(x.ev_cw, x.stream));
  OnStream _os(x, x.stream2);
  do_Y_front(x, false, x.ev_cw);
  DFMI_HIP(hipEventRecord(x.ev_join, x.stream2));
}
void do_U_Y(Ctx& x) {
  if (!step_overlap(x)) { do_U(x); do_Y(x); return; }
  do_U_Y_fork(x);
  do_U(x);
  DFMI_HIP(hipStreamWaitEvent(x.stream, x.ev_join, 0));
  do_Y_back(x);
}
void do_E_back(Ctx& x) {
  Matrix& A = x.mE;
  solve_bicgstab(x, "E", 1, nullptr, A.lower, 0, A.upper, 0, A.diag, 0, A.source, 0, A.ic, A.bc, 0, "he", x.f("he"), 0,
                 x.solver["E"]);
  e_post_solve(x);
}
void do_E(Ctx& x) {
  e_assemble(x);
  do_E_back(x);
}
// UEqn, YEqn, EEqn with the overlap above and one more: the EEqn scheme terms (K's limited weights from the
// UEqn's K, the cubic correction of hDiffCorrFlux from the YEqn preparation) read nothing the Y solve writes,
// so they run on the side stream after both while the main stream solves the species; the rest of the
// assembly needs the solved Y (the thermo's boundary energy gradient) and follows the Y solve
void do_U_Y_E(Ctx& x) {
  if (!step_overlap(x)) { do_U_Y(x); do_E(x); return; }
  do_U_Y_fork(x);
  do_U(x);
  DFMI_HIP(hipEventRecord(x.ev_u, x.stream));
  {
    OnStream _os(x, x.stream2);
    DFMI_HIP(hipStreamWaitEvent(x.stream2, x.ev_u, 0));
    e_assemble_front(x);
    DFMI_HIP(hipEventRecord(x.ev_e, x.stream2));
  }
  DFMI_HIP(hipStreamWaitEvent(x.stream, x.ev_join, 0));
  do_Y_back(x);
  DFMI_HIP(hipStreamWaitEvent(x.stream, x.ev_e, 0));
  e_assemble_back(x);
  do_E_back(x);
}
// correctThermo split in two: the state the pressure corrector reads (T, he, psi, rho) on the main stream, and the
// transport (mu, alpha, rhoD, hai) -- read by nothing before the next time step's equations -- on the side stream,
// where it runs beside the p solves (their coarse AMG levels leave most CUs idle). Its inputs (T, Y) are not
// written again in the step; the main stream waits for it at the end of the step. Option thermo.split (0: fused).
bool do_thermo_split(Ctx& x) {
  if (!step_overlap(x) || !x.on("thermo.split") || species_generic(x) || !x.stream2) {
    thermo_correct(x, false);
    return false;
  }
  thermo_correct(x, false, 1);
  DFMI_HIP(hipEventRecord(x.ev_th, x.stream));
  {
    OnStream _os(x, x.stream2);
    DFMI_HIP(hipStreamWaitEvent(x.stream2, x.ev_th, 0));
    thermo_correct(x, false, 2);
    DFMI_HIP(hipEventRecord(x.ev_tr, x.stream2));
  }
  return true;
}
void do_p(Ctx& x) {
  p_assemble(x);
  Matrix& A = x.mP;
  solve_pcg(x, "p", A.lower, A.upper, A.diag, A.source, A.ic, A.bc, "p", x.f("p"), x.f("boundary_p"), x.solver["p"]);
  p_post_solve(x);
}

}  // namespace

extern "C" {

const char* dfmi_version(void) { return "dfmi 0.1 (gfx950)"; }

int dfmi_last_error(char* buf, int len) {
  if (buf && len > 0) std::snprintf(buf, len, "%s", g_err.c_str());
  return (int)g_err.size();
}

int dfmi_create(dfmi_ctx** out, int device) {
  return guard([&] {
    DFMI_CHECK(out, "null output pointer");
    int n = 0;
    DFMI_HIP(hipGetDeviceCount(&n));
    DFMI_CHECK(device >= 0 && device < n, "device " + std::to_string(device) + " not available (" + std::to_string(n) + " devices)");
    DFMI_HIP(hipSetDevice(device));
    auto* c = new dfmi_ctx();
    c->x.device = device;
    DFMI_HIP(hipStreamCreateWithFlags(&c->x.stream, hipStreamNonBlocking));
    *out = c;
  });
}

int dfmi_destroy(dfmi_ctx* ctx) {
  return guard([&] {
    if (!ctx) return;
    DFMI_HIP(hipSetDevice(ctx->x.device));
    (void)hipStreamSynchronize(ctx->x.stream);
    hipStream_t s = ctx->x.stream;
    delete ctx;
    (void)hipStreamDestroy(s);
  });
}

int dfmi_set_constant_values(dfmi_ctx* ctx, int num_cells, int num_total_cells, int num_surfaces,
                             int num_boundary_surfaces, int num_patches, int num_proc_surfaces,
                             const int* patch_size, int num_species, double rdelta_t) {
  return guard([&] {
    Ctx& x = ctx->x;
    DFMI_CHECK(num_cells > 0 && num_surfaces >= 0 && num_boundary_surfaces >= 0 && num_patches >= 0, "bad sizes");
    // the FV kernels are instantiated for 2..16 species (a larger count fails there, loudly); the DNN
    // surrogate path alone runs up to 64 (BASELINE config 4: GRI-53)
    DFMI_CHECK(num_species >= 2 && num_species <= 64, "num_species must be in [2,64]");
    DFMI_CHECK(rdelta_t > 0, "rdelta_t must be positive");
    x.C = num_cells; x.Ctot = num_total_cells; x.F = num_surfaces; x.B = num_boundary_surfaces; x.P = num_patches;
    x.nproc_faces = num_proc_surfaces; x.S = num_species; x.rdt = rdelta_t;
    x.psize.assign(patch_size, patch_size + num_patches);
    x.pkind.assign(num_patches, 0);
    x.cyc_nbr.assign(num_patches, -1);
    x.peer.assign(num_patches, -1);
    x.have_sizes = true;
  });
}

int dfmi_set_cyclic_info(dfmi_ctx* ctx, const int* cyclic_neighbor) {
  return guard([&] {
    Ctx& x = ctx->x;
    DFMI_CHECK(x.have_sizes, "call dfmi_set_constant_values first");
    x.cyc_nbr.assign(cyclic_neighbor, cyclic_neighbor + x.P);
  });
}

int dfmi_set_constant_indexes(dfmi_ctx* ctx, const int* owner, const int* neighbour, const int* proc_rows,
                              const int* proc_cols, int global_offset) {
  (void)proc_rows;   // global CSR row ids are an AmgX concern; the halo pairs patches by procCols
  return guard([&] {
    Ctx& x = ctx->x;
    DFMI_CHECK(x.have_sizes, "call dfmi_set_constant_values first");
    x.global_offset = global_offset;
    x.h_proc_cols.assign(proc_cols, proc_cols + x.nproc_faces);
    const int C = x.C, F = x.F;
    x.h_own.assign(owner, owner + F);
    x.h_nei.assign(neighbour, neighbour + F);
    std::vector<int> ownStart(C + 1, 0), nbrCnt(C + 1, 0);
    for (int f = 0; f < F; ++f) {
      const int o = owner[f], n = neighbour[f];
      DFMI_CHECK(o >= 0 && o < C && n >= 0 && n < C && o < n, "face " + std::to_string(f) + ": owner/neighbour out of range or owner >= neighbour");
      DFMI_CHECK(f == 0 || owner[f - 1] < o || (owner[f - 1] == o && neighbour[f - 1] < n),
                 "faces are not in upper-triangular order (sorted by owner, then neighbour)");
      ownStart[o + 1]++;
      nbrCnt[n + 1]++;
    }
    for (int c = 0; c < C; ++c) { ownStart[c + 1] += ownStart[c]; nbrCnt[c + 1] += nbrCnt[c]; }
    // face storage: owner-slot order (k-th owned face of c at k*C + c) when at most 3 faces per cell
    // are owned or the padding stays small; OpenFOAM order otherwise
    int kmax = 0;
    for (int c = 0; c < C; ++c) kmax = std::max(kmax, ownStart[c + 1] - ownStart[c]);
    x.fslot = F > 0 && (kmax <= 3 || (long)kmax * C <= (long)F + F / 4);
    x.Fs = x.fslot ? kmax * C : F;
    x.h_fst.resize(F);
    for (int f = 0; f < F; ++f) x.h_fst[f] = x.fslot ? (f - ownStart[owner[f]]) * C + owner[f] : f;
    std::vector<int> own_s(std::max(x.Fs, 1), -1), nei_s(std::max(x.Fs, 1), -1);
    for (int f = 0; f < F; ++f) { own_s[x.h_fst[f]] = owner[f]; nei_s[x.h_fst[f]] = neighbour[f]; }
    std::vector<int> nbrFace(std::max(F, 1)), pos(nbrCnt.begin(), nbrCnt.end() - 1);
    for (int f = 0; f < F; ++f) nbrFace[pos[neighbour[f]]++] = x.h_fst[f];   // ascending face order per cell
    x.own.upload(own_s, x.stream);
    x.nei.upload(nei_s, x.stream);
    x.ownStart.upload(ownStart, x.stream);
    x.nbrStart.upload(nbrCnt, x.stream);
    x.nbrFace.upload(nbrFace, x.stream);
    DFMI_HIP(hipStreamSynchronize(x.stream));
    x.have_topo = true;
  });
}

int dfmi_init_constant_fields_internal(dfmi_ctx* ctx, const double* sf, const double* mag_sf, const double* weight,
                                       const double* delta_coeffs, const double* volume, const double* mesh_distance) {
  // mesh_distance (C[nei] - C[own]) is the d the limited schemes' limiter reads (LimitedScheme::calcLimiter);
  // the reference's GPU path uploads it for its disabled limitedLinear (dfMatrixOpBase.cu:2540-2600)
  return guard([&] {
    Ctx& x = ctx->x;
    DFMI_CHECK(x.have_topo, "call dfmi_set_constant_indexes first");
    const long F = x.F, Fs = x.Fs;
    std::vector<double> soa(3 * std::max(Fs, 1L), 0.0), ms(std::max(Fs, 1L), 0.0), ww(std::max(Fs, 1L), 0.0),
        dd(std::max(Fs, 1L), 0.0), mdv(3 * std::max(Fs, 1L), 0.0);
    for (long f = 0; f < F; ++f) {   // AoS -> SoA, OpenFOAM face order -> face storage
      const long s = x.h_fst[f];
      for (int k = 0; k < 3; ++k) soa[k * Fs + s] = sf[f * 3 + k];
      if (mesh_distance) for (int k = 0; k < 3; ++k) mdv[k * Fs + s] = mesh_distance[f * 3 + k];
      ms[s] = mag_sf[f]; ww[s] = weight[f]; dd[s] = delta_coeffs[f];
    }
    x.md.upload(mdv, x.stream);
    x.Sf.upload(soa, x.stream);
    x.magSf.upload(ms, x.stream);
    x.w.upload(ww, x.stream);
    x.dc.upload(dd, x.stream);
    x.V.upload(volume, x.C, x.stream);
    DFMI_HIP(hipStreamSynchronize(x.stream));
    x.have_md = mesh_distance != nullptr;
    x.have_geom = true;
  });
}

int dfmi_init_constant_fields_boundary(dfmi_ctx* ctx, const double* bsf, const double* bmag, const double* bdelta,
                                       const double* bweight, const int* bface_cell, const int* ptype_calc,
                                       const int* ptype_extrap) {
  return guard([&] {
    Ctx& x = ctx->x;
    DFMI_CHECK(x.have_geom, "call dfmi_init_constant_fields_internal first");
    const long B = x.B;
    for (int p = 0; p < x.P; ++p) {
      const int t = ptype_calc[p];
      x.pkind[p] = (t == CYCLIC) ? 1 : (bc_proc(t) ? 2 : 0);
    }
    x.h_bfc.assign(bface_cell, bface_cell + B);
    std::vector<double> soa(3 * B);
    for (long b = 0; b < B; ++b) for (int k = 0; k < 3; ++k) soa[k * B + b] = bsf[b * 3 + k];
    x.bSf.upload(soa.empty() ? std::vector<double>{0.0} : soa, x.stream);
    x.bmagSf.upload(bmag, B, x.stream);
    x.bdc.upload(bdelta, B, x.stream);
    x.bw.upload(bweight, B, x.stream);
    build_boundary_topology(x);
    allocate_fields(x);
    set_ptype(x, "calculated", ptype_calc);
    set_ptype(x, "extrapolated", ptype_extrap);
    DFMI_HIP(hipStreamSynchronize(x.stream));
    x.have_bgeom = true;
    maybe_setup_halo(x);
  });
}

int dfmi_set_patch_types(dfmi_ctx* ctx, const char* field, const int* patch_type) {
  return guard([&] {
    Ctx& x = ctx->x;
    DFMI_CHECK(x.have_bgeom, "call dfmi_init_constant_fields_boundary first");
    std::string f(field);
    static const char* ok[] = {"U", "p", "he", "K", "Y", "T", "rho"};
    DFMI_CHECK(std::find_if(std::begin(ok), std::end(ok), [&](const char* s) { return f == s; }) != std::end(ok),
               "unknown patch-type field '" + f + "'");
    for (int p = 0; p < x.P; ++p) {
      const int t = patch_type[p];
      DFMI_CHECK(t >= 0 && t <= 12 && t != COUPLED, "patch " + std::to_string(p) + ": unsupported boundary condition code " + std::to_string(t));
      DFMI_CHECK(t != WAVE_TRANSMISSIVE || f == "p", "waveTransmissive is supported for p (the 1D flame's outlet)");
      DFMI_CHECK(t != INLET_OUTLET || f == "U" || f == "p" || f == "Y" || f == "K",
                 "inletOutlet is supported for U, p, Y and K (energy needs its own mixed form)");
      DFMI_CHECK((x.pkind[p] == 1) == (t == CYCLIC) && (x.pkind[p] == 2) == bc_proc(t),
                 "patch " + std::to_string(p) + ": field '" + f + "' type disagrees with the mesh patch kind");
      DFMI_CHECK(t != GRADIENT_ENERGY || f == "he", "gradientEnergy is an energy boundary condition (field 'he')");
      DFMI_CHECK(t != FIXED_ENERGY || f == "he", "fixedEnergy is an energy boundary condition (field 'he')");
    }
    set_ptype(x, f, patch_type);
    DFMI_HIP(hipStreamSynchronize(x.stream));
  });
}

int dfmi_init_boundary_delta(dfmi_ctx* ctx, const double* boundary_delta) {
  return guard([&] {
    Ctx& x = ctx->x;
    DFMI_CHECK(x.have_bgeom, "call dfmi_init_constant_fields_boundary first");
    const long B = x.B;
    std::vector<double> soa(3 * std::max(B, 1L), 0.0);
    for (long b = 0; b < B; ++b) for (int k = 0; k < 3; ++k) soa[k * B + b] = boundary_delta[b * 3 + k];
    x.bdv.upload(soa, x.stream);
    DFMI_HIP(hipStreamSynchronize(x.stream));
    x.have_bdelta = true;
  });
}

// "limitedLinear01 1" -> (kind, k); a leading "Gauss" accepted (system/fvSchemes divSchemes syntax)
static void parse_scheme(const std::string& term, const std::string& text, int& kind, double& k) {
  std::vector<std::string> tok;
  std::string cur;
  for (char ch : text + " ") {
    if (ch == ' ' || ch == '\t') { if (!cur.empty()) tok.push_back(cur); cur.clear(); }
    else cur += ch;
  }
  if (!tok.empty() && tok[0] == "Gauss") tok.erase(tok.begin());
  DFMI_CHECK(!tok.empty(), term + ": empty scheme");
  const std::string& n = tok[0];
  k = 1.0;
  if (n == "upwind") kind = SCH_UPWIND;
  else if (n == "linear") kind = SCH_LINEAR;
  else if (n == "cubic") kind = SCH_CUBIC;
  else if (n == "limitedLinear" || n == "limitedLinear01" || n == "limitedLinearV") {
    kind = n == "limitedLinear" ? SCH_LL : n == "limitedLinear01" ? SCH_LL01 : SCH_LLV;
    DFMI_CHECK(tok.size() == 2, term + ": " + n + " needs its coefficient k");
    char* end = nullptr;
    k = std::strtod(tok[1].c_str(), &end);
    DFMI_CHECK(end && *end == 0 && k >= 0 && k <= 1, term + ": limitedLinear coefficient must be a number in [0, 1]");
    return;
  } else throw Error("dfmi: " + term + ": unsupported scheme '" + text + "'");
  DFMI_CHECK(tok.size() == 1, term + ": unexpected arguments in '" + text + "'");
}

int dfmi_set_scheme(dfmi_ctx* ctx, const char* term, const char* scheme) {
  return guard([&] {
    Ctx& x = ctx->x;
    // the patch kinds (processor patches) are known only after the boundary initialisation
    DFMI_CHECK(x.have_bgeom, "call dfmi_init_constant_fields_boundary before dfmi_set_scheme");
    const std::string t(term ? term : ""), s(scheme ? scheme : "");
    int kind;
    double k;
    parse_scheme(t, s, kind, k);
    if (t == "div(phi,Yi_h)") {
      DFMI_CHECK(kind == SCH_UPWIND || kind == SCH_LL || kind == SCH_LL01, t + ": upwind, limitedLinear or limitedLinear01");
      x.sch.yh = kind; x.sch.k_yh = k;
    } else if (t == "div(phi,K)") {
      DFMI_CHECK(kind != SCH_CUBIC, t + ": upwind, linear, limitedLinear or limitedLinear01");
      x.sch.K = kind; x.sch.k_K = k;
    } else if (t == "div(hDiffCorrFlux)") {
      DFMI_CHECK(kind == SCH_LINEAR || kind == SCH_CUBIC, t + ": linear or cubic");
      x.sch.hD = kind;
    } else if (t == "div(phi,U)") {
      DFMI_CHECK(kind == SCH_LINEAR || kind == SCH_LLV, t + ": linear or limitedLinearV");
      bool proc = false;
      for (int p : x.pkind) proc |= p == 2;
      DFMI_CHECK(kind == SCH_LINEAR || !proc, t + ": limited schemes on decomposed meshes (processor patches) are not supported");
      x.sch.U = kind; x.sch.k_U = k;
    } else throw Error("dfmi: unknown scheme term '" + t + "' (div(phi,Yi_h), div(phi,K), div(hDiffCorrFlux), div(phi,U))");
  });
}

int dfmi_set_traversal(dfmi_ctx* ctx, const int* order) {
  return guard([&] {
    Ctx& x = ctx->x;
    DFMI_CHECK(x.have_sizes, "call dfmi_set_constant_values first");
    if (!order) { x.trav.release(); return; }
    std::vector<char> seen(x.C, 0);
    for (int t = 0; t < x.C; ++t) {
      DFMI_CHECK(order[t] >= 0 && order[t] < x.C && !seen[order[t]], "traversal order is not a permutation of the cells");
      seen[order[t]] = 1;
    }
    x.trav.upload(order, x.C, x.stream);
    DFMI_HIP(hipStreamSynchronize(x.stream));
  });
}

int dfmi_set_patch_param(dfmi_ctx* ctx, const char* field, int patch, const char* name, double value) {
  return guard([&] {
    Ctx& x = ctx->x;
    DFMI_CHECK(x.have_bgeom, "call dfmi_init_constant_fields_boundary first");
    DFMI_CHECK(patch >= 0 && patch < x.P, "patch index out of range");
    const std::string f(field), n(name);
    DFMI_CHECK(f == "p" && n == "gamma", "patch parameters: ('p', 'gamma') of waveTransmissive");
    std::vector<double> g(x.B);
    DFMI_HIP(hipMemcpy(g.data(), x.f("boundary_p_gamma"), x.B * sizeof(double), hipMemcpyDeviceToHost));
    for (int i = 0; i < x.psize[patch]; ++i) g[x.poff[patch] + i] = value;
    DFMI_HIP(hipMemcpy(x.f("boundary_p_gamma"), g.data(), x.B * sizeof(double), hipMemcpyHostToDevice));
  });
}

int dfmi_set_inert_index(dfmi_ctx* ctx, int inert_index) {
  return guard([&] {
    DFMI_CHECK(inert_index >= 0 && inert_index < ctx->x.S, "inert index out of range");
    ctx->x.inert = inert_index;
  });
}

int dfmi_thermo_set_coeffs(dfmi_ctx* ctx, int S, const double* W, const double* nasa, const double* visc,
                           const double* cond, const double* bdiff) {
  return guard([&] {
    Ctx& x = ctx->x;
    DFMI_CHECK(x.have_sizes && S == x.S, "thermo species count differs from num_species");
    Thermo& t = x.thermo;
    t.S = S;
    t.W.assign(W, W + S); t.nasa.assign(nasa, nasa + 15 * S); t.visc.assign(visc, visc + 5 * S);
    t.cond.assign(cond, cond + 5 * S); t.bdiff.assign(bdiff, bdiff + 5 * S * S);
    t.vc1.resize(S * S); t.vc2.resize(S * S);
    for (int i = 0; i < S; ++i) for (int j = 0; j < S; ++j) {   // init_const_coeff_ptr (dfThermo.cu:22-52)
      t.vc1[i * S + j] = std::pow((1 + W[i] / W[j]), -0.5);
      t.vc2[i * S + j] = std::pow(W[j] / W[i], 0.25);
    }
    thermo_upload(x);
    DFMI_HIP(hipStreamSynchronize(x.stream));
  });
}

int dfmi_thermo_load(dfmi_ctx* ctx, const char* path) {
  std::vector<double> all;
  int S = 0;
  int rc = guard([&] {
    std::ifstream in(path, std::ios::binary);
    DFMI_CHECK(in.good(), std::string("cannot open thermo coefficient file ") + path);
    in.read(reinterpret_cast<char*>(&S), sizeof(int));
    DFMI_CHECK(S > 0 && S <= 64, "bad species count in thermo file");
    const size_t n = S + 15 * S + 5 * S + 5 * S + 5 * S * S;
    all.resize(n);
    in.read(reinterpret_cast<char*>(all.data()), n * sizeof(double));
    DFMI_CHECK((size_t)in.gcount() == n * sizeof(double), "truncated thermo coefficient file");
  });
  if (rc) return rc;
  const double* p = all.data();
  return dfmi_thermo_set_coeffs(ctx, S, p, p + S, p + 16 * S, p + 21 * S, p + 26 * S);
}

int dfmi_set_field(dfmi_ctx* ctx, const char* name, const double* host, long count, int layout) {
  return guard([&] { copy_field(ctx->x, name, host, count, layout, true); });
}
int dfmi_get_field(dfmi_ctx* ctx, const char* name, double* host, long count, int layout) {
  return guard([&] { copy_field(ctx->x, name, host, count, layout, false); });
}

int dfmi_pre_time_step(dfmi_ctx* ctx) { return guard([&] { require_ready(ctx->x); copy_old(ctx->x); }); }
int dfmi_post_time_step(dfmi_ctx* ctx) { return guard([&] { require_ready(ctx->x); }); }
int dfmi_rho_process(dfmi_ctx* ctx) { return guard([&] { require_ready(ctx->x); rho_process(ctx->x, false); }); }
int dfmi_U_process(dfmi_ctx* ctx) { return guard([&] { require_ready(ctx->x); do_U(ctx->x); }); }
int dfmi_Y_process(dfmi_ctx* ctx) {
  return guard([&] {
    require_ready(ctx->x);
    ctx->x.dnn.prepared = false;   // a compaction left by an interrupted time step belongs to an old T
    do_Y(ctx->x);
    if (ctx->x.chem.mode == 1) chem_check(ctx->x);   // the Y solve's polls have passed the chemistry
  });
}
int dfmi_E_process(dfmi_ctx* ctx) { return guard([&] { require_ready(ctx->x); do_E(ctx->x); }); }
int dfmi_p_process(dfmi_ctx* ctx) { return guard([&] { require_ready(ctx->x); do_p(ctx->x); }); }
int dfmi_U_get_HbyA(dfmi_ctx* ctx) { return guard([&] { require_ready(ctx->x); u_hbya(ctx->x); }); }
int dfmi_thermo_correct(dfmi_ctx* ctx) { return guard([&] { require_ready(ctx->x); thermo_correct(ctx->x, false); }); }
int dfmi_thermo_update_energy(dfmi_ctx* ctx) { return guard([&] { require_ready(ctx->x); thermo_correct(ctx->x, true); }); }
int dfmi_thermo_update_rho(dfmi_ctx* ctx) { return guard([&] { require_ready(ctx->x); thermo_rho_from_psi(ctx->x); }); }
int dfmi_thermo_psip0(dfmi_ctx* ctx) { return guard([&] { require_ready(ctx->x); thermo_psip0(ctx->x); }); }
int dfmi_thermo_correct_psip_rho(dfmi_ctx* ctx) { return guard([&] { require_ready(ctx->x); thermo_correct_psip_rho(ctx->x); }); }

// dfLowMachFoam.C:284-531 with nOuterCorrectors = 1 (the configuration every reference GPU case uses)
int dfmi_time_step(dfmi_ctx* ctx, int n_corr) {
  return guard([&] {
    Ctx& x = ctx->x;
    require_ready(x);
    // a step that throws records no end mark: restart the timer's ring so no reported interval spans two steps
    struct TimerReset {
      StepTimer& t;
      bool done = false;
      ~TimerReset() { if (!done) t.used = 0; }
    } treset{x.steptimer};
    if (x.steptimer.on && x.steptimer.used == 0) x.steptimer.mark(x.stream);
    x.dnn.prepared = false;         // never reuse a compaction of an earlier (failed) step
    copy_old(x);                    // preTimeStep
    if (x.chem.mode == 2) dnn_prepare(x);   // reacting cells of this step's T (read after the UEqn polls)
    rho_process(x, false);          // rhoEqn (first PIMPLE iteration)
    do_U_Y_E(x);                    // UEqn, YEqn, EEqn (one rank: the chemistry and YEqn assembly beside the
                                    // UEqn, the EEqn assembly beside the Y solve)
    const bool tsplit = do_thermo_split(x);   // correctThermo (the transport half beside the p solves)
    for (int i = 0; i < n_corr; ++i) {   // pEqn_GPU.H
      // rho = psi p: the first corrector's is what correctThermo just wrote (the same product of the same p and psi,
      // halo included); psip0 = psi p feeds only correctPsipRho, skipped below (the field is not updated here)
      if (i > 0) thermo_rho_from_psi(x);
      u_hbya(x);
      // a later corrector may precondition with this step's first hierarchy; with amg.reuse_steps = k > 1 the first
      // corrector too, with the operators of up to k - 1 steps before (rebuilt when they are that old)
      const int keep = (int)x.opt("amg.reuse_steps");
      x.amg.reuse_ok = i > 0 || (keep > 1 && x.amg.ready && x.amg.age > 0 && x.amg.age < keep);
      if (i == 0) x.amg.age = x.amg.reuse_ok ? x.amg.age + 1 : 1;
      do_p(x);
      x.amg.reuse_ok = false;
      // pEqn_GPU.H ends with thermo.correctPsipRho() and the rhoEqn; both write rho, which the next statement here
      // -- rho = psi p at the next corrector's start, or after the loop (dfLowMachFoam.C:517) -- overwrites before
      // anything reads it (the oracle's time_step runs them: the fields agree bitwise). dfmi_thermo_correct_psip_rho /
      // dfmi_rho_process keep them for callers that read rho in between.
    }
    thermo_rho_from_psi(x);         // rho = thermo.rho() (dfLowMachFoam.C:517)
    if (x.chem.mode == 1) chem_check(x);   // the p solves' polls have already passed the chemistry
    if (tsplit) DFMI_HIP(hipStreamWaitEvent(x.stream, x.ev_tr, 0));
    if (x.steptimer.on) x.steptimer.mark(x.stream);
    treset.done = true;
  });
}

int dfmi_step_timer(dfmi_ctx* ctx, int on) {
  return guard([&] {
    Ctx& x = ctx->x;
    DFMI_HIP(hipStreamSynchronize(x.stream));
    x.steptimer.on = on != 0;
    x.steptimer.used = 0;
  });
}

int dfmi_step_times(dfmi_ctx* ctx, double* ms, int n, int* got) {
  return guard([&] {
    Ctx& x = ctx->x;
    DFMI_HIP(hipStreamSynchronize(x.stream));
    const StepTimer& t = x.steptimer;
    // intervals between consecutive marks still in the ring: the last min(used, CAP) - 1 of them
    const size_t kept = std::min(t.used, StepTimer::CAP);
    const int have = kept > 1 ? (int)kept - 1 : 0;
    const size_t m0 = t.used - kept;
    for (int i = 0; i < have && i < n; ++i) {
      float v = 0;
      DFMI_HIP(hipEventElapsedTime(&v, t.at(m0 + i), t.at(m0 + i + 1)));
      ms[i] = v;
    }
    if (got) *got = have;
  });
}

// correct_boundary_conditions_{scalar,vector} of one named field (dfMatrixOpBase.cu:2402-2491)
int dfmi_correct_boundary(dfmi_ctx* ctx, const char* field) {
  return guard([&] {
    Ctx& x = ctx->x;
    require_ready(x);
    std::string f(field);
    if (f == "Y") k_bc_correct(x, "Y", x.f("Y"), x.f("boundary_Y"), x.S);
    else if (f == "U") k_bc_correct(x, "U", x.f("U"), x.f("boundary_U"), 3);
    else if (f == "p" || f == "he" || f == "T" || f == "rho" || f == "K") k_bc_correct(x, f.c_str(), x.f(f), x.f("boundary_" + f), 1);
    else throw Error("dfmi_correct_boundary: unsupported field '" + f + "'");
    halo_fields(x, {f.c_str()});
    DFMI_HIP(hipStreamSynchronize(x.stream));
  });
}

int dfmi_comm_timer(dfmi_ctx* ctx, int on) {
  return guard([&] {
    Ctx& x = ctx->x;
    DFMI_HIP(hipStreamSynchronize(x.stream));
    x.comm.reset();
    x.comm.on = on != 0;
    x.comm.tag.clear();
  });
}

int dfmi_comm_report(dfmi_ctx* ctx, char* buf, int len, int* needed) {
  return guard([&] {
    const std::string r = comm_report(ctx->x);
    if (needed) *needed = (int)r.size() + 1;
    if (buf && len > 0) std::snprintf(buf, len, "%s", r.c_str());
  });
}

int dfmi_kernel_timer(dfmi_ctx* ctx, const char* kernels) {
  return guard([&] {
    Ctx& x = ctx->x;
    DFMI_HIP(hipStreamSynchronize(x.stream));
    KernelTimer& k = x.ktimer;
    k.targets.clear(); k.rec.clear(); k.used = 0;
    std::string s(kernels ? kernels : ""), cur;
    for (char ch : s + ",") {
      if (ch == ',') { if (!cur.empty()) k.targets.push_back(cur); cur.clear(); }
      else if (ch != ' ') cur += ch;
    }
  });
}

int dfmi_kernel_time_named(dfmi_ctx* ctx, const char* kernel, double* total_ms, int* launches) {
  return guard([&] {
    Ctx& x = ctx->x;
    DFMI_HIP(hipStreamSynchronize(x.stream));
    KernelTimer& k = x.ktimer;
    int t = -1;
    for (size_t i = 0; i < k.targets.size(); ++i) if (k.targets[i] == kernel) t = (int)i;
    DFMI_CHECK(t >= 0, std::string("kernel '") + kernel + "' is not armed");
    double tot = 0;
    int n = 0;
    for (size_t r = 0; r < k.rec.size() && 2 * r + 1 < k.used; ++r) {
      if (k.rec[r] != t) continue;
      float ms = 0;
      DFMI_HIP(hipEventElapsedTime(&ms, k.pool[2 * r], k.pool[2 * r + 1]));
      tot += ms;
      ++n;
    }
    *total_ms = tot;
    *launches = n;
  });
}

int dfmi_kernel_time(dfmi_ctx* ctx, double* total_ms, int* launches) {
  return guard([&] {
    DFMI_CHECK(!ctx->x.ktimer.targets.empty(), "no kernel armed");
    const std::string first = ctx->x.ktimer.targets[0];
    if (dfmi_kernel_time_named(ctx, first.c_str(), total_ms, launches)) throw Error(g_err);
  });
}

int dfmi_sync(dfmi_ctx* ctx) { return guard([&] { DFMI_HIP(hipStreamSynchronize(ctx->x.stream)); }); }

int dfmi_hbm_copy_peak(dfmi_ctx* ctx, double gib, int reps, double* gbs) {
  return guard([&] {
    DFMI_CHECK(gib > 0 && reps > 0 && gbs, "bad arguments");
    *gbs = hbm_copy_gbs(ctx->x, (size_t)(gib * (1ull << 30)), reps);
  });
}

int dfmi_assemble(dfmi_ctx* ctx, const char* eqn) {
  return guard([&] {
    Ctx& x = ctx->x;
    require_ready(x);
    std::string e(eqn);
    if (e == "rho") {
      if (!x.fields.count("dbg_rho_diag")) { alloc_field(x, "dbg_rho_diag", x.C, 1, false); alloc_field(x, "dbg_rho_source", x.C, 1, false); }
      rho_process(x, true);
    } else if (e == "U") {
      if (!x.fields.count("dbg_gradU")) alloc_field(x, "dbg_gradU", x.C, 9, false);
      u_assemble(x);
    } else if (e == "Y") {
      if (!x.fields.count("dbg_gradY")) alloc_field(x, "dbg_gradY", x.C, 3 * x.S, false);
      y_prep(x); y_assemble(x);
    } else if (e == "Y_ell") {        // production: fused assembly straight into the solver rows
      YWs _yw(x);
      std::vector<int> map;
      for (int s = 0; s < x.S; ++s) if (s != x.inert) map.push_back(s);
      double *val, *dS, *rhs;
      bicg_layout(x, (int)map.size(), &val, &dS, &rhs);
      y_prep(x);
      y_assemble_ell(x, x.ell.W, (long)x.C + x.H, val, dS, rhs);
    } else if (e == "Y_ell_ref") {    // LDU assembly folded by the generic solver gather
      YWs _yw(x);
      y_prep(x); y_assemble(x);
      bicg_rows_from_ldu_Y(x);
    } else if (e == "E") { conv_weights(x); e_assemble(x); }   // EEqn inspected on its own: fresh div(phi,Yi_h) weights
    else if (e == "p") p_assemble(x);
    else if (e == "HbyA") u_hbya(x);
    else if (e == "p_post") p_post_solve(x);
    else if (e == "Y_post") y_post_solve(x);
    else throw Error("unknown equation '" + e + "'");
    DFMI_HIP(hipStreamSynchronize(x.stream));
  });
}

int dfmi_get_matrix(dfmi_ctx* ctx, const char* eqn, const char* part, double* host, long count) {
  return guard([&] {
    Ctx& x = ctx->x;
    std::string e(eqn), p(part);
    Matrix* A = e == "U" ? &x.mU : e == "Y" ? &x.mY : e == "E" ? &x.mE : e == "p" ? &x.mP : nullptr;
    DFMI_CHECK(A, "unknown equation '" + e + "'");
    DevBuf<double>* b = p == "lower" ? &A->lower : p == "upper" ? &A->upper : p == "diag" ? &A->diag :
                        p == "source" ? &A->source : p == "source_solve" ? &A->source_solve :
                        p == "internal_coeffs" ? &A->ic : p == "boundary_coeffs" ? &A->bc : nullptr;
    DFMI_CHECK(b && b->p, "unknown matrix part '" + p + "'");
    if (p == "lower" || p == "upper") {   // face storage -> OpenFOAM face order, per system
      const long ns = (long)(b->n / std::max(x.Fs, 1));
      DFMI_CHECK(count == ns * x.F, "matrix part size mismatch: expected " + std::to_string(ns * x.F));
      std::vector<double> st(b->n);
      DFMI_HIP(hipMemcpyAsync(st.data(), b->p, b->n * sizeof(double), hipMemcpyDeviceToHost, x.stream));
      DFMI_HIP(hipStreamSynchronize(x.stream));
      for (long s = 0; s < ns; ++s)
        for (long f = 0; f < x.F; ++f) host[s * x.F + f] = st[s * x.Fs + x.h_fst[f]];
      return;
    }
    DFMI_CHECK((size_t)count == b->n, "matrix part size mismatch: expected " + std::to_string(b->n));
    DFMI_HIP(hipMemcpyAsync(host, b->p, count * sizeof(double), hipMemcpyDeviceToHost, x.stream));
    DFMI_HIP(hipStreamSynchronize(x.stream));
  });
}

int dfmi_get_solver_rows(dfmi_ctx* ctx, const char* eqn, const char* part, double* host, long count) {
  return guard([&] {
    Ctx& x = ctx->x;
    DFMI_CHECK(std::string(eqn) == "Y", "solver rows are inspectable for the YEqn batch only");
    YWs _yw(x);
    bicg_rows_get(x, x.S - 1, part, host, count);
  });
}

int dfmi_set_solver(dfmi_ctx* ctx, const char* eqn, int max_iter, double tol, double abs_tol) {
  return guard([&] {
    std::string e(eqn);
    DFMI_CHECK(e == "U" || e == "Y" || e == "E" || e == "p", "unknown equation '" + e + "'");
    DFMI_CHECK(max_iter > 0 && tol >= 0 && abs_tol >= 0, "bad solver controls");
    SolverCfg& c = ctx->x.solver[e];
    c.max_iter = max_iter; c.tol = tol; c.abs_tol = abs_tol;
  });
}

int dfmi_chem_set_mechanism(dfmi_ctx* ctx, int n_reactions, const int* idata, const int* irs, const double* ddata) {
  return guard([&] {
    DFMI_CHECK(ctx->x.have_sizes, "call dfmi_set_constant_values first");
    chem_upload(ctx->x, n_reactions, idata, irs, ddata);
  });
}

int dfmi_chem_set_options(dfmi_ctx* ctx, int mode, double rtol, double atol, double T_min) {
  return guard([&] {
    DFMI_CHECK(mode >= 0 && mode <= 2, "chemistry mode must be 0 (off), 1 (ODE) or 2 (DNN)");
    DFMI_CHECK(rtol > 0 && atol > 0, "chemistry tolerances must be positive");
    Chem& c = ctx->x.chem;
    c.mode = mode; c.rtol = rtol; c.atol = atol; c.Tmin = T_min;
  });
}

int dfmi_dnn_set_model(dfmi_ctx* ctx, int n_modules, int n_layers, const int* dims, const float* params,
                       const double* x_mu, const double* x_std, const double* y_mu, const double* y_std,
                       double T_react, double dt_infer) {
  return guard([&] {
    DFMI_CHECK(ctx->x.have_sizes && ctx->x.inert >= 0, "set sizes and the inert index first");
    dnn_upload(ctx->x, n_modules, n_layers, dims, params, x_mu, x_std, y_mu, y_std, T_react, dt_infer);
  });
}

int dfmi_dnn_load_model(dfmi_ctx* ctx, const char* path, double T_react, double dt_infer) {
  std::vector<char> raw;
  int rc = guard([&] {
    DFMI_CHECK(path, "null path");
    std::ifstream in(path, std::ios::binary);
    DFMI_CHECK(in.good(), std::string("cannot open DF-ODENet model file ") + path);
    raw.assign(std::istreambuf_iterator<char>(in), std::istreambuf_iterator<char>());
  });
  if (rc) return rc;
  int nmod = 0, nl = 0;
  std::vector<int> dims;
  std::vector<double> xmu, xstd, ymu, ystd;
  std::vector<float> params;
  rc = guard([&] {
    size_t o = 0;
    auto take = [&](void* dst, size_t n) {
      DFMI_CHECK(o + n <= raw.size(), std::string("truncated DF-ODENet model file ") + path);
      std::memcpy(dst, raw.data() + o, n);
      o += n;
    };
    char magic[8];
    take(magic, 8);
    DFMI_CHECK(std::memcmp(magic, "DFMIDNN1", 8) == 0, std::string(path) + ": not a packed DF-ODENet file (DFMIDNN1)");
    take(&nmod, 4);
    take(&nl, 4);
    DFMI_CHECK(nmod >= 1 && nmod <= 63 && nl >= 1 && nl <= 8, std::string(path) + ": bad module / layer counts");
    dims.resize(nl + 1);
    take(dims.data(), 4 * dims.size());
    size_t np = 0;
    for (int l = 0; l < nl; ++l) {
      DFMI_CHECK(dims[l] > 0 && dims[l] <= 65536 && dims[l + 1] > 0 && dims[l + 1] <= 65536, std::string(path) + ": bad widths");
      np += (size_t)dims[l] * dims[l + 1] + dims[l + 1];
    }
    xmu.resize(dims[0]); xstd.resize(dims[0]); ymu.resize(nmod); ystd.resize(nmod);
    take(xmu.data(), 8 * xmu.size()); take(xstd.data(), 8 * xstd.size());
    take(ymu.data(), 8 * ymu.size()); take(ystd.data(), 8 * ystd.size());
    params.resize(np * nmod);
    take(params.data(), 4 * params.size());
    DFMI_CHECK(o == raw.size(), std::string(path) + ": trailing bytes after the parameters");
  });
  if (rc) return rc;
  return dfmi_dnn_set_model(ctx, nmod, nl, dims.data(), params.data(), xmu.data(), xstd.data(), ymu.data(), ystd.data(),
                            T_react, dt_infer);
}

int dfmi_dnn_infer(dfmi_ctx* ctx, int* n_reacting) {
  return guard([&] {
    Ctx& x = ctx->x;
    require_ready(x);
    x.dnn.prepared = false;         // standalone inference: compact on the current T
    dnn_solve(x, "rho");
    DFMI_HIP(hipStreamSynchronize(x.stream));
    if (n_reacting) *n_reacting = x.dnn.last_reacting;
  });
}

int dfmi_dnn_stats(dfmi_ctx* ctx, int* n_reacting, double* gemm_flops) {
  return guard([&] {
    Dnn& d = ctx->x.dnn;
    if (n_reacting) *n_reacting = d.last_reacting;
    if (gemm_flops) *gemm_flops = d.gemm_flops;
    d.gemm_flops = 0;
  });
}

int dfmi_chem_info(dfmi_ctx* ctx, int* generated) {
  return guard([&] { *generated = ctx->x.chem.generated; });
}

int dfmi_chem_solve(dfmi_ctx* ctx, double dt) {
  return guard([&] {
    Ctx& x = ctx->x;
    require_ready(x);
    DFMI_CHECK(dt > 0, "chemistry time step must be positive");
    chem_solve(x, dt, "rho");
    DFMI_HIP(hipStreamSynchronize(x.stream));
    chem_check(x);
  });
}

int dfmi_zero_d_step(dfmi_ctx* ctx, double dt, int n_steps) {
  return guard([&] {
    Ctx& x = ctx->x;
    require_ready(x);
    DFMI_CHECK(dt > 0 && n_steps >= 1, "0D step: dt and n_steps must be positive");
    x.dnn.prepared = false;
    // no host synchronisation inside the loop: the steps' launches queue back to back (one round trip per step
    // bounded config 1 at ~0.1 ms/step), the chemistry's failure counter sums over the batch and is read once
    Chem& h = x.chem;
    if (h.mode == 1) {
      if (h.fail.n == 0) h.fail.alloc(1);
      DFMI_HIP(hipMemsetAsync(h.fail.p, 0, sizeof(int), x.stream));
      h.batch = true;
    }
    struct BatchEnd {
      Chem& h;
      ~BatchEnd() { h.batch = false; }
    } bend{h};
    for (int i = 0; i < n_steps; ++i) zero_d_step(x, dt);
    if (h.mode == 1) {
      h.batch = false;
      chem_fail_snapshot(x);
      chem_check(x);
    }
    DFMI_HIP(hipStreamSynchronize(x.stream));
  });
}

int dfmi_chem_set_max_steps(dfmi_ctx* ctx, int max_steps) {
  return guard([&] {
    DFMI_CHECK(max_steps > 0, "max_steps must be positive");
    ctx->x.chem.max_steps = max_steps;
  });
}

int dfmi_amg_info(dfmi_ctx* ctx, int max_levels, int* n_levels, int* cells, int* width) {
  return guard([&] {
    const Amg& a = ctx->x.amg;
    *n_levels = (int)a.lv.size();
    for (int l = 0; l < (int)a.lv.size() && l < max_levels; ++l) { cells[l] = a.lv[l].n; width[l] = a.lv[l].W; }
    if (a.global && (int)a.lv.size() < max_levels) {   // the agglomerated level, listed last
      cells[a.lv.size()] = a.ng; width[a.lv.size()] = a.wg;
      *n_levels += 1;
    }
  });
}

int dfmi_row_classes(dfmi_ctx* ctx, int* n) {
  return guard([&] { *n = ctx->x.ell.ready ? ctx->x.ell.ncls : 0; });
}

int dfmi_hex_dims(dfmi_ctx* ctx, int* nx, int* ny, int* nz) {
  return guard([&] {
    const bool on = ctx->x.ell.ready;
    *nx = on ? ctx->x.hex[0] : 0; *ny = on ? ctx->x.hex[1] : 0; *nz = on ? ctx->x.hex[2] : 0;
  });
}

int dfmi_set_option(dfmi_ctx* ctx, const char* key, double value) {
  return guard([&] {
    Ctx& x = ctx->x;
    (void)x.opt(key);   // throws for an unknown key
    const std::string k(key);
    // keys read when the AMG hierarchy (amg_setup) or the solver rows (build_ell) are built; every other key is
    // read at each call (amg.reuse per p solve, pcg.* / fv.* / chem.* / dnn.* per launch)
    static const char* structural_keys[] = {"amg.omega", "amg.overcorrection", "amg.coarsest_sweeps",
                                            "amg.coarsest_size", "amg.presweeps", "amg.pairwise_passes_l0",
                                            "amg.pairwise_passes", "amg.precision", "amg.padded", "amg.tail",
                                            "amg.halo_l0", "amg.global_coarse", "solver.even_odd", "solver.small",
                                            "solver.row_classes"};
    bool structural = false;
    for (const char* s : structural_keys) structural |= k == s;
    DFMI_CHECK(!structural || (!x.amg.ready && !x.ell.ready),
               "dfmi_set_option: '" + k + "' shapes the solver structures; set it before the first solve");
    x.opts[k] = value;
  });
}

int dfmi_get_option(dfmi_ctx* ctx, const char* key, double* value) {
  return guard([&] { *value = ctx->x.opt(key); });
}

int dfmi_set_preconditioner(dfmi_ctx* ctx, const char* eqn, const char* name) {
  return guard([&] {
    std::string e(eqn), n(name);
    DFMI_CHECK(e == "U" || e == "Y" || e == "E" || e == "p", "unknown equation '" + e + "'");
    DFMI_CHECK(n == "jacobi" || (n == "amg" && e == "p"), "preconditioner must be 'jacobi' or ('amg' for p)");
    ctx->x.solver[e].precond = n == "amg" ? 1 : 0;
  });
}

int dfmi_solver_stats(dfmi_ctx* ctx, const char* eqn, int* iters, double* res0, double* rel) {
  return guard([&] {
    const SolveStats st = solve_stats(ctx->x, eqn);
    if (iters) *iters = st.iters;
    if (res0) *res0 = st.res0;
    if (rel) *rel = st.res;
  });
}

int dfmi_solver_work(dfmi_ctx* ctx, const char* eqn, double* iters, int reset) {
  return guard([&] {
    const double v = solver_work(ctx->x, eqn, reset != 0);
    if (iters) *iters = v;
  });
}

namespace {
void set_comm(Ctx& x, int nranks, int rank, const int* neighb) {
  DFMI_CHECK(x.have_sizes, "call dfmi_set_constant_values first");
  DFMI_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank / nranks");
  x.nranks = nranks;
  x.rank = rank;
  x.peer.assign(neighb, neighb + x.P);
  // overlapped solver halos: the option halo.overlap (read per solve); the environment sets its default here
  const char* e = std::getenv("DFMI_HALO_OVERLAP");
  if (e && !x.opts.count("halo.overlap")) x.opts["halo.overlap"] = std::atoi(e) != 0 ? 1.0 : 0.0;
}
// the exchange lists need the boundary topology: built now, or at the end of
// dfmi_init_constant_fields_boundary (every rank reaches both points in the same order)
void maybe_setup_halo(Ctx& x) {
  if (!x.halo || !x.have_bgeom) return;
  int nproc = 0;
  for (int p = 0; p < x.P; ++p) if (x.pkind[p] == 2) nproc += x.psize[p];
  DFMI_CHECK(nproc == x.nproc_faces, "num_proc_surfaces differs from the processor patch sizes");
  halo_setup(x);
}
}  // namespace

int dfmi_set_comm_info(dfmi_ctx* ctx, const void* uid, int nranks, int rank, const int* neighb) {
  return guard([&] {
    Ctx& x = ctx->x;
    set_comm(x, nranks, rank, neighb);
    halo_init_rccl(x, uid, nranks, rank);
    maybe_setup_halo(x);
  });
}

int dfmi_set_comm_local(dfmi_ctx* ctx, int hub_id, int nranks, int rank, const int* neighb) {
  return guard([&] {
    Ctx& x = ctx->x;
    set_comm(x, nranks, rank, neighb);
    halo_init_local(x, hub_id, nranks, rank);
    maybe_setup_halo(x);
  });
}

int dfmi_get_unique_id(void* out) { return guard([&] { rccl_unique_id(out); }); }

int dfmi_renumber_cells(int num_cells, const double* cell_centres, int num_faces, const int* owner,
                        const int* neighbour, const char* method, int* new_to_old) {
  return guard([&] { renumber_cells(num_cells, cell_centres, num_faces, owner, neighbour, method, new_to_old); });
}

int dfmi_renumber_faces(int num_cells, int num_faces, const int* owner, const int* neighbour,
                        const int* cell_new_to_old, int* face_new_to_old, int* new_owner, int* new_neighbour,
                        int* flipped) {
  return guard([&] {
    renumber_faces(num_cells, num_faces, owner, neighbour, cell_new_to_old, face_new_to_old, new_owner, new_neighbour,
                   flipped);
  });
}

}  // extern "C"
