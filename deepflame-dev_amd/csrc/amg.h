// amg.h -- aggregation-AMG preconditioner state (amg.hip)
#pragma once
#include "dfmi_common.h"
#include <array>
#include <map>

namespace dfmi {

struct Ctx;

struct AmgLevel {
  int n = 0, W = 0;
  DevBuf<int> col;                      // [W][n] (levels >= 1; level 0 uses the solver ELL)
  DevBuf<int> agg, mstart, members;     // fine -> coarse map, coarse -> fine member lists (to level+1)
  DevBuf<int> gstart, gsrc;             // Galerkin contribution lists building level+1
  // per-solve operator (levels >= 1; level 0 in fp32 mode: a rounded copy of the solver ELL) and
  // work vectors, in the preconditioner's precision (one of the two sets is allocated)
  DevBuf<double> val, D, b, x, r, xo;
  DevBuf<float> fval, fD, fb, fx, fr, fxo;
  DevBuf<double> r2, zt;                // level 0 with l0_sweeps > 1: second residual, post-sweep ping-pong
  DevBuf<float> fr2;
};

// Precision of the V-cycle (amg.precision). fp32 (default) keeps every level's operator and work vectors in single
// precision (AmgX's mixed mode: preconditioner in float, Krylov iteration in double); the outer PCG
// residuals, dot products and solution stay fp64, so the attainable accuracy is unchanged and only
// the preconditioner's HBM traffic halves. amg.precision = 64 keeps the whole hierarchy in double.
struct Amg {
  bool ready = false;
  bool reuse_ok = false;   // set by dfmi_time_step for its later correctors (option amg.reuse)
  int age = 0;             // time steps since the V-cycle's operators were last rebuilt (option amg.reuse_steps)
  bool fp32 = true;
  double omega = 0.9;
  double overcorr = 1.35;  // coarse-correction scaling (plain aggregation under-corrects; 1 = plain V-cycle)
  int coarse_sweeps = 8;
  int l0_sweeps = 1;       // weighted-Jacobi sweeps before and after the coarse correction on level 0
  bool padded = false;     // levels 1 .. L-2 in aligned groups of 8 per aggregate (pad_levels)
  bool tail = false;       // levels L-2 and L-1 of the fp32 V-cycle in one workgroup (k_vtail)
  int coarsest = 4096;
  std::vector<AmgLevel> lv;
  // Agglomerated coarsest level (several ranks; amg.global_coarse = 1, off by default: measured no fewer
  // p-iterations). The rank-local hierarchies stop at
  // coarsest / nranks cells; every rank's coarsest cells are gathered into ONE global level of ng = nranks x
  // nmax cells (rank r's cell I at r nmax + I, padding rows with a unit diagonal) whose operator includes the
  // couplings across processor faces (level-0 halo coefficients summed per pair of coarsest aggregates).
  // Per solve the ranks all-gather their packed rows; per V-cycle their coarsest right-hand sides, and every
  // rank smooths the identical global level redundantly (k_coarsest) -- the role of AmgX's consolidated
  // coarse levels (src_gpu/AmgXSolver.cu:184-266) in place of block-Jacobi across ranks.
  // level 0 with its processor couplings (several ranks; amg.halo_l0 = 0: off): the first sweep's residual and
  // the post-sweep include the halo columns (the PCG residual and diagonal exchanged, the prolongated
  // correction exchanged before the post-sweep) instead of dropping them (block-Jacobi)
  bool halo_l0 = false;
  // level 0 read face-wise (FaceOp; one rank, hex box, symmetric p: solve_pcg sets dfo each solve, the fp32
  // copies of its face and slot coefficients are rounded here) instead of from the ELL values
  bool face = false;
  FaceOp<double> dfo;
  FaceOp<float> ffo;
  DevBuf<float> fup, fbc;
  const double* dS_full = nullptr;        // this solve's level-0 diagonal incl. the exchanged halo entries [C + H]
  DevBuf<double> hy;                      // prolongated level-0 iterate incl. halo [C + H]
  bool global = false;
  int nmax = 0, ng = 0, wc = 0, we = 0, wg = 0, nloc = 0;
  DevBuf<int> g_col;                      // [wg][ng] global columns
  DevBuf<int> e_start, e_src;             // external sums: (row I, slot e) -> level-0 ELL sources k C + c
  DevBuf<double> g_send, g_recv;          // packed rows: own nmax (wg + 1), all ng (wg + 1)
  DevBuf<double> g_bs, g_bg;              // coarsest right-hand side: own nmax, all ng
  DevBuf<double> g_val, g_D, g_x;         // global operator / solution in the V-cycle precision (f64 ...)
  DevBuf<float> g_fval, g_fD, g_fx;       // (... or f32)
};

// The hierarchy as plain pointers (one workgroup runs the whole V-cycle of a small system in
// linsolve.hip). Level 0's operator is the solver ELL (f64) or its rounded copy (f32); its right-hand
// side is the PCG residual, so b[0] is unused.
constexpr int AMG_MAXL = 12;
template <class T> struct AmgView {
  int L = 0;
  int n[AMG_MAXL], W[AMG_MAXL];
  const int* col[AMG_MAXL];
  const T* val[AMG_MAXL];
  const T* D[AMG_MAXL];
  T* b[AMG_MAXL];
  T* x[AMG_MAXL];
  T* r[AMG_MAXL];
  T* xo[AMG_MAXL];
  const int* agg[AMG_MAXL];
  const int* mstart[AMG_MAXL];
  const int* members[AMG_MAXL];
  T omega, sc;
  int sweeps;
};
AmgView<float> amg_view_f32(Ctx& x, const int* col0);
AmgView<double> amg_view_f64(Ctx& x, const double* val0, const double* D0, const int* col0);

// The PCG stop test (linsolve.hip k_cg_spmv: ||r|| <= tol ||r0|| or <= abs_tol) evaluated by the V-cycle's
// first launch after the fused update, from the same partials in the same order, so a converged solve skips
// its last V-cycle; k_cg_spmv of iteration `it` then finds the flag set and returns. The recorded residual and
// iteration count are the ones k_cg_spmv would record.
struct CgStop {
  Red rr;               // the update's r.r partials
  double* scal;         // PCG scalars (4 res0, 5 res, 6 active, 7 iters); nullptr: no test
  int it;               // the PCG iteration the test belongs to
  double tol, abs_tol;
};

void amg_setup(Ctx& x);
void amg_galerkin(Ctx& x, const double* val0, const double* D0);
// z = M^-1 r with block partials of r.z written to partial[0 .. nblk) (grid of `nblk` blocks); every
// kernel returns at once when *active == 0 (a converged solve; nullptr: always run)
void amg_apply(Ctx& x, const double* val0, const double* D0, ColView col0, const double* r, double* z,
               double* partial, int nblk, const double* active = nullptr, bool l0_done = false,
               const CgStop& stop = CgStop{});
// the level-0 first sweep (x0, residual) can be written by the PCG update kernel instead (linsolve.hip:
// k_cg_x_smooth): fp32 V-cycle, launch-per-level path, one pre-sweep, at least two levels
bool amg_l0_fusable(const Ctx& x);

}  // namespace dfmi
