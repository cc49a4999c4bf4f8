// amg.h -- aggregation-AMG preconditioner state (amg.hip)
#pragma once
#include "dfmi_common.h"

namespace dfmi {

struct Ctx;

struct AmgLevel {
  int n = 0, W = 0;
  DevBuf<int> col;                      // [W][n] (levels >= 1; level 0 uses the solver ELL)
  DevBuf<double> val, D;                // per-solve coarse operator (levels >= 1)
  DevBuf<int> agg, mstart, members;     // fine -> coarse map, coarse -> fine member lists (to level+1)
  DevBuf<int> gstart, gsrc;             // Galerkin contribution lists building level+1
  DevBuf<double> b, x, r, xo;           // work vectors
};

struct Amg {
  bool ready = false;
  double omega = 0.85;
  int coarse_sweeps = 8;
  int coarsest = 4096;
  std::vector<AmgLevel> lv;
};

void amg_setup(Ctx& x);
void amg_galerkin(Ctx& x, const double* val0, const double* D0);
// z = M^-1 r with block partials of r.z written to partial[0 .. nblk) (grid of `nblk` blocks)
void amg_apply(Ctx& x, const double* val0, const double* D0, const int* col0, const double* r, double* z,
               double* partial, int nblk);

}  // namespace dfmi
