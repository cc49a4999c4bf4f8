// dfmi_ctx.h -- the device-resident database (the MI355X counterpart of dfMatrixDataBase,
// reference src_gpu/dfMatrixDataBase.H:97-324) plus per-equation workspaces.
//
// HBM layout (all fp64 values SoA, int32 indices):
//   cells: scalar [C]; vector [3][C]; tensor [9][C]; species [S][C] (species-major)
//   faces: [F]; vectors [3][F]
//   boundary slots: [B] in OpenFOAM patch order, processor patches take 2n slots
//                   [neighbour values n | patch-internal values n] (createGPUSolver.H:118-123)
// Topology for deterministic cell gathers (no FP atomics anywhere):
//   ownStart[C+1]           faces owned by c are [ownStart[c], ownStart[c+1]) (upper-triangular order)
//   nbrStart[C+1], nbrFace  faces whose neighbour is c, ascending face index (losort)
// Face STORAGE: every face array lives in "owner-slot" order when the mesh allows it (at most a few
// faces owned per cell, e.g. hex meshes: 3): the k-th face owned by cell c at k*C + c. A wavefront of
// consecutive cells then reads and writes its k-th owned faces as one contiguous run (OpenFOAM order
// interleaves each cell's 3 faces: stride-3 partial lines that the L2 evicts between the three
// visits), and a cell's neighbour-side faces are the owned faces of consecutive cells too. Padding
// slots have own = -1. The API keeps OpenFOAM face order: face fields and lower/upper are mapped
// through h_fst (face -> storage) at the boundary. Meshes with many owned faces per cell keep face order.
//   cbStart[C+1], cbSlot    primary boundary slots of c, ascending slot index
// Visiting nbrFace, then own faces, then cbSlot is exactly OpenFOAM's sequential face order.
#pragma once
#include "dfmi_common.h"
#include "amg.h"
#include <map>
#include <memory>

namespace dfmi {

constexpr int SCODE_PAD = -1;   // row-class source code of a padding entry (esrc PAD)

struct MeshView {
  int C, F, B, S;
  const int *own, *nei, *ownStart, *nbrStart, *nbrFace, *cbStart, *cbSlot, *bfc, *partner;
  int fslot;                // face storage in owner-slot order (k*C + c) rather than OpenFOAM order
  const int8_t* sprim;   // 1 = primary slot (owner side), 0 = processor [internal n] slot
  const double *Sf, *magSf, *w, *dc, *V, *bSf, *bmagSf, *bw, *bdc;
  const int *ecol, *esrc;   // solver gather rows [W][C] (linsolve.hip build_ell): the face loops read them
  int W;
  // row classes (ColView): column offsets and source codes per class [ncls][W]; a source code is
  // 2 kslot + own (face storage kslot * C + owner cell), SCODE_PAD for padding, CEXPL: read esrc
  const uint8_t* ecls;
  const int *ectab, *estab;
  double rdt;
  // hex box in blockMesh order (cell c = i + nx (j + ny k), internal faces towards +x/+y/+z in owner-slot
  // storage, build_ell checked every row against it): the face walk computes face and neighbour indices
  // instead of loading them (each_face<-1>); hx = 0: not such a mesh
  int hx, hy, hz;
  const int* trav;          // optional traversal order of the per-cell gather kernels (thread t -> cell)
  const double *md, *bdv;   // C[nei] - C[own] [3][F] (face storage) and patch delta vectors [3][B] (limited schemes)
  // even-odd solver layout (Ctx::Ell::eo): row index of cell c in the BiCGStab rows / vectors (first the
  // colour-0 cells, then colour-1, each ascending); nullptr: natural order. Only the writers of the
  // BiCGStab rows (k_ell_build for U/E, k_y_assemble_ell) read it.
  const int* eopos;
};

// entry k of cell c's gather row: column j and coefficient source e (2 f + own for the face at storage f,
// -(b + 1) for boundary slot b, INT_MIN padding), from the row class cl (ecls_of) or the explicit arrays
__device__ __forceinline__ int ecls_of(const MeshView& m, int c) { return m.ecls ? (int)m.ecls[c] : -1; }
__device__ __forceinline__ void erow(const MeshView& m, int cl, int k, int c, int& j, int& e) {
  const long C = m.C;
  if (cl >= 0) {
    const int o = m.ectab[cl * m.W + k], sc = m.estab[cl * m.W + k];
    j = o != CEXPL ? c + o : m.ecol[k * C + c];
    if (sc == SCODE_PAD) e = CEXPL;   // == INT_MIN, the ELL padding code
    else if (sc != CEXPL) e = 2 * ((sc >> 1) * (int)C + ((sc & 1) ? c : j)) + (sc & 1);
    else e = m.esrc[k * C + c];
    return;
  }
  j = m.ecol[k * C + c];
  e = m.esrc[k * C + c];
}

// interpolation / convection schemes of the terms the reference GPU path hard-wires (dfmi_set_scheme;
// dfmi/schemes.py): div(phi,Yi_h), div(phi,K), div(hDiffCorrFlux)
enum SchemeKind { SCH_UPWIND = 0, SCH_LINEAR = 1, SCH_LL = 2, SCH_LL01 = 3, SCH_CUBIC = 4, SCH_LLV = 5 };
struct Schemes {
  int yh = SCH_UPWIND, K = SCH_LINEAR, hD = SCH_LINEAR, U = SCH_LINEAR;
  double k_yh = 1.0, k_K = 1.0, k_U = 1.0;
};

struct Field {
  DevBuf<double> buf;
  long n = 0;       // values per component (device storage; faces: Fs)
  int ncomp = 1;
  bool boundary = false;
  bool face = false;  // internal-face field: API order F, device storage Fs (Ctx::h_fst)
};

// one assembled fvMatrix (LDU + boundary coefficients), reference storage convention
struct Matrix {
  int nsys = 1;                 // species batch for Y
  DevBuf<double> lower, upper, diag, source, ic, bc;
  DevBuf<double> source_solve;  // U only: source incl. -grad(p)
};

struct SolverCfg {
  int max_iter = 20;
  double tol = 1e-5;           // relative to the initial residual (AmgX RELATIVE_INI, amgxUOptions)
  double abs_tol = 0.0;
  int precond = 0;             // 0 Jacobi, 1 aggregation AMG (p only)
};

struct SolveStats { int iters = 0; double res0 = 0, res = 0; };

struct Thermo {
  int S = 0;
  std::vector<double> W, nasa, visc, cond, bdiff, vc1, vc2;
  DevBuf<double> dW, drW, dnasa, dvisc, dcond, dbdiff, dvc1, dvc2;   // drW = 1 / W
  std::vector<double> hc;        // Hf298_i / W_i [J/kg]: the heat-release weights (dfChemistryModel.C:335-338)
  DevBuf<double> dhc;
  // species-minor copies for the cooperative S > 16 kernel (lanes own consecutive species i, so a
  // coefficient load over a group is one contiguous run): nasa [15][S], bdiff [j][5][i], vc [j][i]
  DevBuf<double> dnasaT, dbdiffT, dvc1T, dvc2T;
  // the same kernel's packed forms: vc1 / vc2 interleaved [j][i][2] (one 16-B load per pair), and, for a symmetric
  // binary-diffusion table, its unique pairs in rotation order [d - 1][i][6] = coefficients of the pair
  // (i, (i + d) mod S), d = 1 .. S / 2, padded to 6 (three 16-B loads)
  DevBuf<double> dvcP, dbdR;
};

struct Halo;   // RCCL processor-patch exchange (halo.hip)

// DF-ODENet surrogate (dnn.hip): S-1 MLPs, fp16 weights per layer [module][out][Kpad], fp32 biases
struct Dnn {
  bool ready = false;
  int nmod = 0;
  std::vector<int> dims, Kp;
  std::vector<DevBuf<_Float16>> W;
  std::vector<DevBuf<float>> b;
  DevBuf<double> xmu, xstd, ymu, ystd;
  double T_react = 610.0, dt = 1e-6;      // unReactT_ (dfChemistrySolver.cu:90), RR divisor (:191)
  int chunk = 65536;                      // reacting cells per inference batch
  int last_reacting = 0;
  double gemm_flops = 0;                  // algorithmic GEMM flops issued since the last query
  DevBuf<int> bc, idx;
  DevBuf<_Float16> x0, h0, h1;
  DevBuf<float> part;           // fused output layer: per-row partial dot products [net][2 N tiles][chunk]
  // reacting-cell count: compacted at the start of the time step (T is frozen until correctThermo) and
  // copied to pinned memory behind an event, read by dnn_solve after the UEqn solve's polls -- no drain
  PinnedBuf<int> nr_host;
  hipEvent_t nr_ev = nullptr;
  bool prepared = false;
  ~Dnn() { if (nr_ev) (void)hipEventDestroy(nr_ev); }
};

// per-cell chemistry (chem.hip): mechanism arrays (dfmi/kinetics.py layout) and integrator controls
struct Chem {
  bool ready = false;
  int mode = 0;                 // 0 off, 1 stiff ODE integration, 2 DNN surrogate
  int R = 0, ndd = 0;
  DevBuf<int> idata, irs;
  DevBuf<double> dd;
  double rtol = 1e-6, atol = 1e-10, Tmin = 0.0;   // CVODE settings of the reference (CanteraTorchProperties)
  int max_steps = 100000;
  int method = 0;               // 0 ROS3 Rosenbrock, 1 linearly-implicit Euler extrapolation
  int generated = 0;            // last solve used a compiled-in mechanism (chem_gen_*.inc): 1 burke9, 2 es80
  int bin = 2;                  // order cells by the previous solve's step count (option chem.binning: 0 natural order, 1 whole mesh, 2 per tile)
  DevBuf<int> perm, bcnt;       // cost-binned cell order; per-block bucket counts / offsets
  std::vector<int> h_idata, h_irs;
  std::vector<double> h_dd;
  DevBuf<int> fail;             // cells of the last solve that hit max_steps (device counter)
  PinnedBuf<int> fail_host;     // its copy, behind fail_ev
  hipEvent_t fail_ev = nullptr;
  bool fail_pending = false;
  bool batch = false;           // dfmi_zero_d_step's loop: the counter sums over the batch, read once at its end
  ~Chem() { if (fail_ev) (void)hipEventDestroy(fail_ev); }
};

// HIP-event timing of one named kernel (dfmi_kernel_timer / dfmi_kernel_time)
struct KernelTimer {
  std::vector<std::string> targets;   // armed kernel names
  std::vector<hipEvent_t> pool;       // pairs (start, end)
  std::vector<int> rec;               // target index of each recorded pair
  size_t used = 0;
  ~KernelTimer() { for (auto e : pool) (void)hipEventDestroy(e); }
  hipEvent_t next() {
    if (used == pool.size()) {
      hipEvent_t e;
      DFMI_HIP(hipEventCreate(&e));
      pool.push_back(e);
    }
    return pool[used++];
  }
};

// Per-step timing (dfmi_step_timer / dfmi_step_times): while armed, dfmi_time_step records an event on the
// context stream before its first step and after every step (no synchronisation), so the bench reads each
// step's duration -- end of step i to end of step i-1 -- and reports their median beside the bracketed mean.
// The events form a ring of CAP marks, so an armed timer holds a bounded number of events however many steps
// run; dfmi_step_times reports the last CAP - 1 intervals. A step that fails resets the ring (its end mark is
// never recorded, and an interval spanning two steps must not be reported).
struct StepTimer {
  static constexpr size_t CAP = 1024;
  bool on = false;
  std::vector<hipEvent_t> ev;         // mark m at ev[m % CAP]: m = 0 before the first armed step, m = i after step i
  size_t used = 0;                    // marks recorded since arming (or since the last failed step)
  ~StepTimer() { for (auto e : ev) (void)hipEventDestroy(e); }
  void mark(hipStream_t s) {
    const size_t slot = used % CAP;
    if (slot == ev.size()) {
      hipEvent_t e;
      DFMI_HIP(hipEventCreate(&e));
      ev.push_back(e);
    }
    DFMI_HIP(hipEventRecord(ev[slot], s));
    ++used;
  }
  hipEvent_t at(size_t m) const { return ev[m % CAP]; }
};

// Communication accounting per exchange point (dfmi_comm_timer / dfmi_comm_report): every transport call
// of a halo exchange (ncclSend/ncclRecv group) or an all-gather, HIP events around it on the stream it is
// issued on (the compute stream, or the halo's comm stream for overlapped exchanges), with the bytes this
// rank sends, keyed by the exchange point that issued it (Ctx::comm.tag, set by the callers: the field
// names of a boundary-field exchange, the solver and its vectors). The reference's counterparts are the
// per-field NCCL groups of dfMatrixOpBase.cu:441-485 / 2402-2491, timed only by its TIME_GPU host ticks.
struct CommStats {
  bool on = false;
  std::string tag;
  struct Entry { long calls = 0; double bytes = 0; std::vector<std::pair<hipEvent_t, hipEvent_t>> ev; };
  std::map<std::string, Entry> pts;
  std::vector<hipEvent_t> pool;
  size_t used = 0;
  hipEvent_t next() {
    if (used == pool.size()) {
      hipEvent_t e;
      DFMI_HIP(hipEventCreate(&e));
      pool.push_back(e);
    }
    return pool[used++];
  }
  void reset() { pts.clear(); used = 0; }
  ~CommStats() { for (auto e : pool) (void)hipEventDestroy(e); }
};

// Implementation options (dfmi_set_option; the role the reference's amgx*Options files and
// CanteraTorchProperties switches play for its solvers): the AMG configuration of the p solver, the solver
// and face-walk choices, the chemistry integrator. Every key and its default is listed here; an unknown key is
// an error. They are read when the structure they shape is built (the AMG hierarchy and the solver rows at
// the first solve) or at each call (everything else).
struct OptDef { const char* key; double def; };
inline const OptDef* option_defs(int& n) {
  static const OptDef d[] = {
    {"amg.omega", 0.9},               // weighted-Jacobi smoothing weight (0.85 -> 0.9: 13 -> 12 p-iterations)
    {"amg.overcorrection", 1.4},      // coarse-correction scaling of the plain-aggregation V-cycle
    {"amg.coarsest_sweeps", 6},       // Jacobi sweeps on the coarsest level (amgxpOptions coarsest_sweeps; 2 in the
                                      // reference's AmgX hierarchy). 1.35 / 8 -> 1.4 / 6: 13.88 -> 13.74 and 13.92 -> 13.81
                                      // ms per step, 3 rounds each in two calls (profiles/r06_ab_misc.txt r06m / r06n)
    {"amg.coarsest_size", 512},       // coarsening stops at this many cells
    {"amg.presweeps", 1},             // level-0 pre- and post-sweeps (amgxpOptions presweeps / postsweeps)
    {"amg.pairwise_passes_l0", 3},    // pairwise-matching passes building level 1 (3: 2x2x2 aggregates; SIZE_2 x 3)
    {"amg.pairwise_passes", 3},       // ... building the levels below
    {"amg.precision", 32},            // 32: V-cycle in fp32 (AmgX mixed mode), 64: fp64
    {"amg.padded", 1},                // coarse levels in aligned groups of 8 per aggregate (one launch per level)
    {"amg.tail", 1},                  // the last two levels in one workgroup launch (k_vtail)
    {"amg.halo_l0", 1},               // several ranks: level 0 keeps its processor couplings
    {"amg.global_coarse", 0},         // several ranks: one agglomerated coarsest level
    {"amg.reuse_steps", 8},           // > 1: the first corrector reuses the V-cycle operators of up to this many - 1
                                      // earlier steps (1: rebuilt every step). 1 -> 8: 13.59 -> 13.42 ms per step, 3
                                      // rounds each, 674 against 678 p system-iterations in 28 steps (r06u)
    {"amg.reuse", 1},                 // later correctors of a time step precondition with the step's first V-cycle
                                      // operators (level-0 fp32 copy, Galerkin levels) instead of rebuilding them
    {"solver.even_odd", 1},           // U/Y/E: BiCGStab on the even-odd Schur complement where the rows 2-colour
    {"solver.small", 1},              // one rank, <= 4096 cells: every solve in one workgroup
    {"solver.row_classes", 1},        // solver rows decoded from one byte per cell where the mesh allows
    {"pcg.face_form", 1},             // one rank, hex box: the p operator read face-wise
    {"pcg.fuse_l0", 1},               // the PCG update fused with the V-cycle's level-0 first sweep
    {"fv.hex_walk", 1},               // hex box in blockMesh order: face and neighbour indices computed
    {"fv.csr_walk", 0},               // assembly faces walked from the CSR lists instead of the gather rows
    {"fv.species_generic", 0},        // the species-chunked YEqn kernels at any species count (S > 16 always)
    {"fv.yprep_brick", 1},            // k_y_prep staging 16x4x4 bricks in LDS (hex walk)
    {"chem.method", 0},               // 0: ROS3 Rosenbrock, 1: linearly-implicit Euler extrapolation
    {"chem.generated", 1},            // compiled-in kinetics when the mechanism's fingerprint matches
    {"chem.binning", 2},              // cells launched in cost-binned order: 1 over the mesh, 2 inside 4096-cell tiles
    {"dnn.tuned_gemm", 1},            // DF-ODENet layers by the shape-tuned kernels (0: k_mlp_gemm for every layer)
    {"thermo.split", 0},              // time step: the transport half of correctThermo on the side stream beside the p solve
                                      // (13.89 -> 13.92 ms per step, 3 rounds each in one call, round 6: not the default)
    {"halo.overlap", 0},              // several ranks: solver halo exchanges on a comm stream while the interior rows run
                                      // (read per solve; DFMI_HALO_OVERLAP sets the default when the communicator is set)
  };
  n = (int)(sizeof(d) / sizeof(d[0]));
  return d;
}

struct Ctx {
  int device = 0;
  std::map<std::string, double> opts;   // dfmi_set_option overrides
  double opt(const char* key) const {
    auto it = opts.find(key);
    if (it != opts.end()) return it->second;
    int n;
    const OptDef* d = option_defs(n);
    for (int i = 0; i < n; ++i) if (std::string(d[i].key) == key) return d[i].def;
    throw Error(std::string("dfmi: unknown option '") + key + "'");
  }
  bool on(const char* key) const { return opt(key) != 0.0; }
  hipStream_t stream = nullptr;
  // sizes (dfMatrixDataBase::setConstantValues, dfMatrixDataBase.cu:114-147)
  int C = 0, Ctot = 0, F = 0, B = 0, P = 0, S = 0, nproc_faces = 0;
  int Fs = 0;                    // face storage size (owner-slot layout: kmax * C; otherwise F)
  bool fslot = false;
  std::vector<int> h_fst;        // OpenFOAM face -> storage index
  double rdt = 0;
  int inert = -1;
  bool have_sizes = false, have_topo = false, have_geom = false, have_bgeom = false;
  bool have_md = false;           // mesh_distance was given (the limited schemes' d; zeros otherwise)
  std::vector<int> psize, poff, pkind, cyc_nbr, peer;   // pkind: 0 plain, 1 cyclic, 2 processor
  std::vector<int> h_bfc, h_own, h_nei;
  // topology
  DevBuf<int> own, nei, ownStart, nbrStart, nbrFace, cbStart, cbSlot, bfc, partner;
  DevBuf<int8_t> sprim;
  // geometry
  DevBuf<double> Sf, magSf, w, dc, V, bSf, bmagSf, bw, bdc;
  DevBuf<double> md, bdv;        // mesh_distance [3][Fs], boundary delta [3][B] (dfmi_init_boundary_delta)
  bool have_bdelta = false;
  Schemes sch;
  DevBuf<int> conv_list, conv_nlist;   // faces whose div(phi,Yi_h) limiter needs gradients (k_conv_w_check)
  // per-field patch types (host, per patch) and per-slot device copies
  std::map<std::string, std::vector<int>> ptype;
  std::map<std::string, DevBuf<int8_t>> stype;
  // fields
  std::map<std::string, Field> fields;
  // matrices
  Matrix mU, mY, mE, mP;
  std::map<std::string, SolverCfg> solver;
  Thermo thermo;
  // scratch
  DevBuf<double> scratch;
  // domain decomposition (halo.cpp): processor patches exchange [neighbour n] slot values
  int nranks = 1, rank = 0, global_offset = 0;
  std::vector<int> h_proc_cols;  // procCols: global id of the cell across each processor face (patch order)
  int H = 0;                     // processor faces = halo values per component
  std::vector<int> h_hidx;       // per boundary slot: halo index of a primary processor slot, else -1
  Halo* halo = nullptr;          // owned; freed by halo_destroy()
  // solver gather (linsolve.hip): per cell W coupling entries, [W][C] (coalesced)
  struct Ell {
    int W = 0;
    bool ready = false;
    DevBuf<int> col;             // column: cell id, or C + halo index for a processor face
    DevBuf<int> src;             // coefficient: 2f = lower[f], 2f+1 = upper[f], -(b+1) = -boundaryCoeffs[b]
    DevBuf<int8_t> bflag;        // [C] 1: the row has a processor (halo) column
    DevBuf<int> brow;            // those rows, ascending
    int nb = 0;
    // row classes (ColView; built when the mesh has <= 255 distinct rows and owner-slot face storage;
    // DFMI_ROW_CLASSES=0: explicit columns everywhere)
    DevBuf<uint8_t> cls;
    DevBuf<int> ctab, stab;
    DevBuf<int> csStart, csSlot, scol;   // coupled slots per cell and their columns (FaceOp)
    int ncls = 0;
    ColView cols() const {
      ColView v;
      v.col = col.p; v.W = W;
      if (ncls > 0) { v.cls = cls.p; v.tab = ctab.p; v.ntab = ncls * W; }
      return v;
    }
    // even-odd (red-black) reduced BiCGStab (linsolve.hip): on a bipartite coupling graph (hex meshes) the
    // rows are stored colour by colour -- colour-0 cells [0, ne), colour-1 cells [ne, C) -- and the solver
    // iterates on the colour-1 Schur complement. eo_pos: cell -> row, eo_cell: row -> cell; eo_col: the
    // ELL columns in row numbering (every entry points into the other colour), with its own row classes
    int eo = 0, ne = 0;
    DevBuf<int> eo_pos, eo_cell, eo_col, eo_ctab;
    DevBuf<uint8_t> eo_cls;
    int eo_ncls = 0;
    std::vector<int> h_eo_pos;
    ColView eo_cols() const {
      ColView v;
      v.col = eo_col.p; v.W = W;
      if (eo_ncls > 0) { v.cls = eo_cls.p; v.tab = eo_ctab.p; v.ntab = eo_ncls * W; }
      return v;
    }
  } ell;
  Amg amg;                       // pressure preconditioner hierarchy (amg.hip)
  Chem chem;
  Dnn dnn;
  struct SolverWs {
    DevBuf<double> buf, scal, red_local, red_all;
    DevBuf<int> sysmap;
    HostRecs poll;                   // convergence records the device posts (linsolve.hip: Poller)
    long long poll_seq = 0;          // records posted so far
  } ws, ws_y;
  // the YEqn batch has its own solver workspace (its rows are assembled while the UEqn solve may still be
  // running on the other stream, dfmi_time_step); linsolve.hip reaches the current one through sws()
  bool ws_is_y = false;
  SolverWs& sws() { return ws_is_y ? ws_y : ws; }
  // side stream of the time step (dfmi_time_step: chemistry + YEqn preparation beside the UEqn) and its events
  hipStream_t stream2 = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_u = nullptr, ev_e = nullptr, ev_cw = nullptr, ev_th = nullptr,
            ev_tr = nullptr;
  // final solver state of the last solve of each equation, copied asynchronously at the end of the
  // solve; dfmi_solver_stats synchronises and reads it (no host sync inside a time step)
  struct StatSnap { PinnedBuf<double> h; int nsys = 0; };
  std::map<std::string, StatSnap> stat_snap;
  std::map<std::string, int> solve_expect;   // iterations of the last solve per equation (linsolve.hip Poller)
  DevBuf<double> work;           // per equation (U, Y, E, p): system-iterations, summed on the device
  KernelTimer ktimer;
  StepTimer steptimer;
  CommStats comm;
  DevBuf<int> trav;   // dfmi_set_traversal: the order threads visit cells in the gather kernels (empty: natural)
  int hex[3] = {0, 0, 0};   // MeshView::hx/hy/hz (build_ell)
  ~Ctx();
  int n_corr = 2;

  MeshView view() const {
    MeshView m;
    m.C = C; m.F = Fs; m.B = B; m.S = S; m.fslot = fslot ? 1 : 0;
    m.own = own; m.nei = nei; m.ownStart = ownStart; m.nbrStart = nbrStart; m.nbrFace = nbrFace;
    m.cbStart = cbStart; m.cbSlot = cbSlot; m.bfc = bfc; m.partner = partner; m.sprim = sprim;
    m.Sf = Sf; m.magSf = magSf; m.w = w; m.dc = dc; m.V = V; m.bSf = bSf; m.bmagSf = bmagSf; m.bw = bw; m.bdc = bdc;
    m.ecol = ell.col; m.esrc = ell.src; m.W = ell.ready ? ell.W : 0;
    // the assembly face loops and the ELL fold read explicit rows (class lookups through the global table
    // measured slower for these latency-bound gathers, round 3)
    m.ecls = nullptr;
    m.ectab = ell.ctab.p; m.estab = ell.stab.p;
    m.rdt = rdt;
    m.trav = trav.n ? trav.p : nullptr;
    m.hx = hex[0]; m.hy = hex[1]; m.hz = hex[2];
    m.md = md.p; m.bdv = bdv.p;
    m.eopos = ell.ready && ell.eo ? ell.eo_pos.p : nullptr;
    return m;
  }
  double* f(const std::string& name) {
    auto it = fields.find(name);
    DFMI_CHECK(it != fields.end(), "unknown field '" + name + "'");
    return it->second.buf.p;
  }
  const int8_t* st(const std::string& field) {
    auto it = stype.find(field);
    DFMI_CHECK(it != stype.end(), "patch types not set for field '" + field + "'");
    return it->second.p;
  }
  // scheme buffers (fv_kernels.hip scheme launchers): 0/1 div(phi,Yi_h) weights (faces / slots), 2/3
  // div(phi,K) weights, 4/5 cubic flux correction of div(hDiffCorrFlux); nullptr where the term keeps
  // the reference GPU path's scheme (upwind / linear / linear); 6/7 div(phi,U) limitedLinearV weights
  const double* sch_w(int i) {
    static const char* names[8] = {"conv_w", "boundary_conv_w", "K_w", "boundary_K_w", "cubic_flux",
                                   "boundary_cubic_flux", "U_w", "boundary_U_w"};
    const bool on = i < 2 ? sch.yh != SCH_UPWIND : i < 4 ? sch.K != SCH_LINEAR : i < 6 ? sch.hD == SCH_CUBIC
                                                                                     : sch.U == SCH_LLV;
    if (!on) return nullptr;
    auto it = fields.find(names[i]);
    DFMI_CHECK(it != fields.end(), std::string("scheme buffer '") + names[i] + "' not computed");
    return it->second.buf.p;
  }
  const std::vector<int>& pt(const std::string& field) {
    auto it = ptype.find(field);
    DFMI_CHECK(it != ptype.end(), "patch types not set for field '" + field + "'");
    return it->second;
  }
};

// The YEqn workspace (Ctx::ws_y) for the scope's solver calls.
struct YWs {
  Ctx& x;
  bool prev;
  explicit YWs(Ctx& c) : x(c), prev(c.ws_is_y) { x.ws_is_y = true; }
  ~YWs() { x.ws_is_y = prev; }
};
// Launches of the scope go to stream s (the launchers all read Ctx::stream).
struct OnStream {
  Ctx& x;
  hipStream_t prev;
  OnStream(Ctx& c, hipStream_t s) : x(c), prev(c.stream) { x.stream = s; }
  ~OnStream() { x.stream = prev; }
};

// Records a start/end event pair around a launch when `name` is the armed kernel.
struct KScope {
  Ctx& x;
  int idx;
  static int match(const std::vector<std::string>& ts, const char* name) {   // template arguments ignored
    if (ts.empty() || !name) return -1;
    while (*name == '(') ++name;
    size_t n = 0;
    while (name[n] && name[n] != '<') ++n;
    for (size_t i = 0; i < ts.size(); ++i)
      if (ts[i].size() == n && ts[i].compare(0, n, name, n) == 0) return (int)i;
    return -1;
  }
  KScope(Ctx& c, const char* name) : x(c), idx(match(c.ktimer.targets, name)) {
    if (idx >= 0) { x.ktimer.rec.push_back(idx); DFMI_HIP(hipEventRecord(x.ktimer.next(), x.stream)); }
  }
  ~KScope() noexcept(false) { if (idx >= 0) DFMI_HIP(hipEventRecord(x.ktimer.next(), x.stream)); }
};

// ---- renumber.cpp (host): cell order for cache-local gathers, faces re-sorted upper-triangular
void renumber_cells(int num_cells, const double* cell_centres, int num_faces, const int* owner, const int* neighbour,
                    const char* method, int* new_to_old);
void renumber_faces(int num_cells, int num_faces, const int* owner, const int* neighbour, const int* cell_new_to_old,
                    int* face_new_to_old, int* new_owner, int* new_neighbour, int* flipped);

// ---- launchers (fv_kernels.hip)
void k_bc_correct(Ctx& x, const char* type_field, double* vf, double* bvf, int ncomp);
void rho_process(Ctx& x, bool write_matrix);
void u_assemble(Ctx& x);
void u_post_solve(Ctx& x);
void u_hbya(Ctx& x);
void p_assemble(Ctx& x);
void p_post_solve(Ctx& x);
void y_prep(Ctx& x, bool weights = true);   // weights = false: the caller formed the div(phi,Yi_h) weights
void y_assemble(Ctx& x);
void y_assemble_ell(Ctx& x, int W, long Ce, double* val, double* dS, double* rhs);
void y_post_solve(Ctx& x);
void e_assemble(Ctx& x);
void e_assemble_front(Ctx& x);   // the scheme terms (independent of the Y solve)
void e_assemble_back(Ctx& x);    // boundary energy gradient, he's boundary values, the matrix
void e_post_solve(Ctx& x);
void conv_weights(Ctx& x);   // div(phi,Yi_h) weights (start of YEqn; EEqn reuses them)
void copy_old(Ctx& x);
void zero_d_step(Ctx& x, double dt);   // df0DFoam loop body for every cell
void thermo_rho_from_psi(Ctx& x);
void thermo_psip0(Ctx& x);
void thermo_correct_psip_rho(Ctx& x);
// thermo.hip
void thermo_upload(Ctx& x);
std::vector<double> heat_of_formation_per_mass(int S, const double* W, const double* nasa);   // hc_i (Qdot weights)
// part 0: the whole update; 1: the state (T, he, psi, rho); 2: the transport (mu, alpha, rhoD, hai) at the
// current T -- the time step runs part 2 on the side stream beside the pressure corrector
void thermo_correct(Ctx& x, bool from_T, int part = 0);
// boundary_heGradient on gradientEnergy slots of he (0 elsewhere)
void thermo_energy_gradient(Ctx& x);
// linsolve.hip
SolveStats solve_bicgstab(Ctx& x, const char* eqn, int nsys, const int* sys_map_host, const double* lower, long lstride,
                          const double* upper, long ustride, const double* diag, long dstride, const double* source,
                          long sstride, const double* ic, const double* bc, long bstride, const char* type_field,
                          double* xsol, long xstride, const SolverCfg& cfg, bool prebuilt = false);
void bicg_layout(Ctx& x, int nsys, double** val, double** dS, double** rhs);
void build_ell(Ctx& x);   // solver gather rows; also the face lists of the assembly kernels
void bicg_rows_from_ldu_Y(Ctx& x);
void bicg_rows_get(Ctx& x, int nsys, const std::string& part, double* host, long count);
bool species_generic(const Ctx& x);   // fv_kernels.hip: chunked kernels for S > 16 (or the option fv.species_generic)
// iterations / initial and final relative residual of the last solve of `eqn` (synchronises)
SolveStats solve_stats(Ctx& x, const std::string& eqn);
// system-iterations of the solves of `eqn` since the last reset (synchronises)
double solver_work(Ctx& x, const std::string& eqn, bool reset);
SolveStats solve_pcg(Ctx& x, const char* eqn, const double* lower, const double* upper, const double* diag,
                     const double* source, const double* ic, const double* bc, const char* type_field, double* xsol,
                     double* bxsol, const SolverCfg& cfg);
// dnn.hip
void dnn_upload(Ctx& x, int nmod, int nlayers, const int* dims, const float* params, const double* xmu,
                const double* xstd, const double* ymu, const double* ystd, double T_react, double dt_infer);
double hbm_copy_gbs(Ctx& x, size_t bytes, int reps);   // measured device copy bandwidth (fv_kernels.hip)
void dnn_prepare(Ctx& x);   // reacting-cell compaction + count read-back, ahead of dnn_solve
void dnn_solve(Ctx& x, const char* rho_field);   // RR scaled by rho_field (reference: d_rho_old, dfYEqn.cu:449)
// chem.hip
void chem_upload(Ctx& x, int R, const int* idata, const int* irs, const double* dd);
// rho_field: the thermo density RR is scaled by (dfChemistryModel.C:771, problem.rhoi = rho_[celli]);
// inside dfmi_time_step that is rho_old (thermo.rho() before this step's rhoEqn), standalone "rho"
void chem_solve(Ctx& x, double dt, const char* rho_field);
void chem_fail_snapshot(Ctx& x);
// throws when the last solve left cells at the step limit (waits on the snapshot event only)
void chem_check(Ctx& x);
// halo.hip
// One exchange point: cell values of each item's components are sent across processor faces and land
// in the receiver's neighbour slots (to_slots) or in the extended vector region [C, C+H) (solver vectors).
struct HaloItem {
  const double* cell;
  double* dst;
  int ncomp;
  long cstride, dstride;
  bool to_slots;
  bool split = false;   // the source vector is stored in the even-odd row order (Ell::eo): send value[eo_pos[cell]]
  int colour = -1;      // split vectors: -1 every processor face; k: only the faces whose sending cell has colour k
                        // (the next half-row pass reads no other halo entries; halo.hip Plan)
};
bool halo_active(const Ctx& x);
void halo_update(Ctx& x, const HaloItem* items, int n);
// overlapped form (solver SpMVs, Ctx::halo_overlap): the exchange runs on the halo's comm stream between
// halo_begin and halo_end; the compute stream meanwhile runs only work that touches no halo entry
bool halo_overlap(const Ctx& x);
void halo_begin(Ctx& x, const HaloItem* items, int n);
void halo_end(Ctx& x);
// the exchange point of the halo / all-gather calls made while it lives (communication accounting)
struct CommTag {
  Ctx& x;
  std::string prev;
  bool set;
  CommTag(Ctx& c, const std::string& t) : x(c), set(c.comm.on) { if (set) { prev = x.comm.tag; x.comm.tag = t; } }
  ~CommTag() { if (set) x.comm.tag = prev; }
};
inline void halo_fields(Ctx& x, const std::vector<const char*>& names) {
  if (!halo_active(x)) return;
  std::string tag;
  if (x.comm.on) {
    tag = "fields";
    for (const char* n : names) { tag += ' '; tag += n; }
  }
  CommTag _ct(x, tag);
  std::vector<HaloItem> it;
  for (const char* n : names) {
    const Field& f = x.fields.at(n);
    const Field& bf = x.fields.at(std::string("boundary_") + n);
    it.push_back({f.buf.p, bf.buf.p, f.ncomp, f.n, bf.n, true});
  }
  halo_update(x, it.data(), (int)it.size());
}
// allgather of `count` doubles per rank: recv[r * count + i]
void halo_allgather(Ctx& x, const double* send, double* recv, long count);
std::string comm_report(Ctx& x);   // JSON of the communication accounting (CommStats)
std::vector<int> halo_peers_of(const Ctx& x);   // neighbour rank of every halo index (processor face)
void halo_set_split(Ctx& x);   // the send map of split (even-odd) vectors, after build_ell decided the layout
void halo_setup(Ctx& x);   // builds the exchange lists after dfmi_set_comm_info / dfmi_set_comm_local
void halo_init_rccl(Ctx& x, const void* uid, int nranks, int rank);
void halo_init_local(Ctx& x, int hub_id, int nranks, int rank);
void rccl_unique_id(void* out);
void halo_destroy(Halo* h);

}  // namespace dfmi
