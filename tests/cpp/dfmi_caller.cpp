// dfmi_caller.cpp -- a compiled C++ host of the drop-in boundary: only include/dfmi.h and -ldfmi.
//
// Mirrors what the OpenFOAM side does through createGPUSolver.H (createGPUBase / createGPU*Eqn /
// createGPUThermo, applications/solvers/dfLowMachFoam/createGPUSolver.H:103-709) and the time loop of
// dfLowMachFoam.C:249-531, on a periodic n^3 hex box generated here (OpenFOAM is not in this image):
// owner/neighbour in upper-triangular order, AoS area vectors, cyclic patches in blockMesh order, the
// reference's thermo_ES80_H2-7-16.txt, a hot kernel in H2/air. Prints one JSON line with the state
// after the steps; exit code 0 only if every call succeeded and the state is physical.
//   usage: dfmi_caller <thermo_ES80_H2-7-16.txt> [n=16] [steps=3]
#include "../../include/dfmi.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace {

dfmi_ctx* g_ctx = nullptr;

void check(int rc, const char* what) {
  if (rc == 0) return;
  char buf[2048];
  dfmi_last_error(buf, sizeof buf);
  std::fprintf(stderr, "%s failed: %s\n", what, buf);
  if (g_ctx) dfmi_destroy(g_ctx);
  std::exit(1);
}

struct Box {
  int n, C, F;
  double h;
  std::vector<int> owner, neighbour;
  std::vector<double> sf, mag, w, dc, vol, md;
  // patches: front(z+) back(z-) left(x-) right(x+) top(y+) down(y-), all cyclic
  std::vector<int> psize, pcyc, bfc;
  std::vector<double> bsf, bmag, bdc, bw;
  int id(int i, int j, int k) const { return i + n * (j + n * k); }
};

Box make_box(int n, double L) {
  Box b;
  b.n = n; b.C = n * n * n; b.h = L / n;
  const double h = b.h, A = h * h;
  for (int c = 0; c < b.C; ++c) {   // faces per owner towards +x, +y, +z (upper-triangular order)
    const int i = c % n, j = (c / n) % n, k = c / (n * n);
    const int nb[3] = {i + 1 < n ? b.id(i + 1, j, k) : -1, j + 1 < n ? b.id(i, j + 1, k) : -1, k + 1 < n ? b.id(i, j, k + 1) : -1};
    for (int d = 0; d < 3; ++d) {
      if (nb[d] < 0) continue;
      b.owner.push_back(c); b.neighbour.push_back(nb[d]);
      for (int e = 0; e < 3; ++e) { b.sf.push_back(e == d ? A : 0.0); b.md.push_back(e == d ? h : 0.0); }
      b.mag.push_back(A); b.w.push_back(0.5); b.dc.push_back(1.0 / h);
    }
  }
  b.F = (int)b.owner.size();
  b.vol.assign(b.C, h * h * h);
  struct Side { int axis, sign; };
  const Side sides[6] = {{2, 1}, {2, -1}, {0, -1}, {0, 1}, {1, 1}, {1, -1}};
  const int partner[6] = {1, 0, 3, 2, 5, 4};
  for (int p = 0; p < 6; ++p) {
    const int ax = sides[p].axis, sg = sides[p].sign, layer = sg > 0 ? n - 1 : 0;
    const int t0 = ax == 0 ? 1 : 0, t1 = ax == 2 ? 1 : 2;   // tangential axes, t0 fastest
    for (int b1 = 0; b1 < n; ++b1)
      for (int b0 = 0; b0 < n; ++b0) {
        int ijk[3];
        ijk[ax] = layer; ijk[t0] = b0; ijk[t1] = b1;
        b.bfc.push_back(b.id(ijk[0], ijk[1], ijk[2]));
        for (int e = 0; e < 3; ++e) b.bsf.push_back(e == ax ? sg * A : 0.0);
        b.bmag.push_back(A); b.bdc.push_back(1.0 / h); b.bw.push_back(0.5);
      }
    b.psize.push_back(n * n);
    b.pcyc.push_back(partner[p]);
  }
  return b;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) { std::fprintf(stderr, "usage: %s thermo_ES80_H2-7-16.txt [n] [steps]\n", argv[0]); return 2; }
  const int n = argc > 2 ? std::atoi(argv[2]) : 16, steps = argc > 3 ? std::atoi(argv[3]) : 3;
  const double L = 6.283185307179586e-3, dt = 1e-6;
  Box b = make_box(n, L);
  const int S = 7, B = 6 * n * n, P = 6;
  const int CYC = 6, CALC = 5, EXTRAP = 8;
  // createGPUBase
  check(dfmi_create(&g_ctx, 0), "dfmi_create");
  check(dfmi_set_constant_values(g_ctx, b.C, b.C, b.F, B, P, 0, b.psize.data(), S, 1.0 / dt), "dfmi_set_constant_values");
  check(dfmi_set_cyclic_info(g_ctx, b.pcyc.data()), "dfmi_set_cyclic_info");
  int none = 0;
  check(dfmi_set_constant_indexes(g_ctx, b.owner.data(), b.neighbour.data(), &none, &none, 0), "dfmi_set_constant_indexes");
  check(dfmi_init_constant_fields_internal(g_ctx, b.sf.data(), b.mag.data(), b.w.data(), b.dc.data(), b.vol.data(), b.md.data()),
        "dfmi_init_constant_fields_internal");
  std::vector<int> cyc(P, CYC), calc(P, CALC), extrap(P, EXTRAP);
  (void)calc; (void)extrap;
  check(dfmi_init_constant_fields_boundary(g_ctx, b.bsf.data(), b.bmag.data(), b.bdc.data(), b.bw.data(), b.bfc.data(),
                                           cyc.data(), cyc.data()), "dfmi_init_constant_fields_boundary");
  // createGPU*Eqn: every field is cyclic on this box
  for (const char* f : {"U", "p", "he", "K", "Y", "T", "rho"}) check(dfmi_set_patch_types(g_ctx, f, cyc.data()), "dfmi_set_patch_types");
  check(dfmi_set_inert_index(g_ctx, 6), "dfmi_set_inert_index");   // ES80: H O H2O OH O2 H2 N2 -> N2
  check(dfmi_thermo_load(g_ctx, argv[1]), "dfmi_thermo_load");     // createGPUThermo
  // initial state: air + H2 at 300 K with a 1500 K kernel, Taylor-Green velocity (AoS, as OpenFOAM)
  const int C = b.C;
  std::vector<double> T(C), p(C, 101325.0), U(3 * C), Y((size_t)S * C, 0.0);
  const double yu[7] = {0, 0, 0, 0, 0.2264, 0.0284, 0.7452}, yb[7] = {0, 0, 0.2548, 0, 0, 0, 0.7452};
  for (int c = 0; c < C; ++c) {
    const int i = c % n, j = (c / n) % n, k = c / (n * n);
    const double x = (i + 0.5) * b.h, y = (j + 0.5) * b.h, z = (k + 0.5) * b.h, Lr = 1e-3;
    const double r2 = std::pow(x - L / 2, 2) + std::pow(y - L / 2, 2) + std::pow(z - L / 2, 2);
    const double pr = std::exp(-r2 / (1.5e-3 * 1.5e-3));
    T[c] = 300.0 + 1500.0 * pr;
    U[3 * c + 0] = 4.0 * std::sin(x / Lr) * std::cos(y / Lr) * std::cos(z / Lr);
    U[3 * c + 1] = -4.0 * std::cos(x / Lr) * std::sin(y / Lr) * std::cos(z / Lr);
    U[3 * c + 2] = 0.0;
    for (int s = 0; s < S; ++s) Y[(size_t)s * C + c] = (1 - pr) * yu[s] + pr * yb[s];
  }
  check(dfmi_set_field(g_ctx, "T", T.data(), C, DFMI_SOA), "set T");
  check(dfmi_set_field(g_ctx, "p", p.data(), C, DFMI_SOA), "set p");
  check(dfmi_set_field(g_ctx, "U", U.data(), C, DFMI_AOS), "set U");
  check(dfmi_set_field(g_ctx, "Y", Y.data(), C, DFMI_SOA), "set Y");
  for (const char* f : {"T", "p", "U", "Y"}) check(dfmi_correct_boundary(g_ctx, f), "dfmi_correct_boundary");
  check(dfmi_thermo_update_energy(g_ctx), "dfmi_thermo_update_energy");
  // phi = interpolate(rho U) & Sf (createPhi): uniform box, w = 1/2; boundary from the cyclic partner
  std::vector<double> rho(C), phi(b.F), bphi(B);
  check(dfmi_get_field(g_ctx, "rho", rho.data(), C, DFMI_SOA), "get rho");
  for (int f = 0; f < b.F; ++f) {
    const int o = b.owner[f], q = b.neighbour[f];
    double a = 0.0;
    for (int e = 0; e < 3; ++e) a += b.sf[3 * f + e] * 0.5 * (rho[o] * U[3 * o + e] + rho[q] * U[3 * q + e]);
    phi[f] = a;
  }
  for (int s = 0; s < B; ++s) {
    const int pt = s / (n * n), i = s % (n * n);
    const int c = b.bfc[s], q = b.bfc[b.pcyc[pt] * n * n + i];
    double a = 0.0;
    for (int e = 0; e < 3; ++e) a += b.bsf[3 * s + e] * 0.5 * (rho[c] * U[3 * c + e] + rho[q] * U[3 * q + e]);
    bphi[s] = a;
  }
  check(dfmi_set_field(g_ctx, "phi", phi.data(), b.F, DFMI_SOA), "set phi");
  check(dfmi_set_field(g_ctx, "boundary_phi", bphi.data(), B, DFMI_SOA), "set boundary_phi");
  std::vector<double> K(C);
  for (int c = 0; c < C; ++c) K[c] = 0.5 * (U[3 * c] * U[3 * c] + U[3 * c + 1] * U[3 * c + 1] + U[3 * c + 2] * U[3 * c + 2]);
  check(dfmi_set_field(g_ctx, "K", K.data(), C, DFMI_SOA), "set K");
  check(dfmi_correct_boundary(g_ctx, "K"), "correct K");
  // time loop (dfLowMachFoam.C:249-531): the whole PIMPLE body per call, nCorr = 2
  double mass0 = 0.0;
  for (int c = 0; c < C; ++c) mass0 += rho[c] * b.vol[c];
  for (int it = 0; it < steps; ++it) check(dfmi_time_step(g_ctx, 2), "dfmi_time_step");
  // write-back (runTime.write(): every written field, not only U and T as the reference GPU path)
  std::vector<double> Tn(C), Yn((size_t)S * C), Un(3 * C);
  check(dfmi_get_field(g_ctx, "T", Tn.data(), C, DFMI_SOA), "get T");
  check(dfmi_get_field(g_ctx, "rho", rho.data(), C, DFMI_SOA), "get rho");
  check(dfmi_get_field(g_ctx, "Y", Yn.data(), C, DFMI_SOA), "get Y");
  check(dfmi_get_field(g_ctx, "U", Un.data(), C, DFMI_AOS), "get U");
  double tmin = 1e30, tmax = -1e30, ysum = 0.0, mass = 0.0;
  bool finite = true;
  for (int c = 0; c < C; ++c) {
    tmin = std::fmin(tmin, Tn[c]); tmax = std::fmax(tmax, Tn[c]);
    double s = 0.0;
    for (int k = 0; k < S; ++k) s += Yn[(size_t)k * C + c];
    ysum = std::fmax(ysum, std::fabs(s - 1.0));
    mass += rho[c] * b.vol[c];
    finite = finite && std::isfinite(Tn[c]) && std::isfinite(Un[3 * c]);
  }
  int iters = 0; double r0 = 0, rel = 0;
  check(dfmi_solver_stats(g_ctx, "p", &iters, &r0, &rel), "dfmi_solver_stats");
  std::printf("{\"cells\": %d, \"steps\": %d, \"T_min\": %.6f, \"T_max\": %.6f, \"max_abs_sumY_minus_1\": %.3e, "
              "\"mass_rel_change\": %.3e, \"p_iters\": %d, \"finite\": %s, \"version\": \"%s\"}\n",
              C, steps, tmin, tmax, ysum, std::fabs(mass - mass0) / mass0, iters, finite ? "true" : "false", dfmi_version());
  check(dfmi_destroy(g_ctx), "dfmi_destroy");
  const bool ok = finite && tmin > 250.0 && tmax < 2500.0 && ysum < 1e-10 && std::fabs(mass - mass0) / mass0 < 1e-6;
  return ok ? 0 : 3;
}
