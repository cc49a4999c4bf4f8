/* collision_q.c -- classical transport cross sections Q(1)*(E), Q(2)*(E) of the 12-6-3 potential
 *     V(r)/eps = 4 [ r^-12 - r^-6 - d r^-3 ]      (r in units of sigma)
 * i.e. Lennard-Jones plus a fixed-orientation dipole-dipole term: the Stockmayer potential as
 * Monchick & Mason (J. Chem. Phys. 35, 1676, 1961) treat it, d = delta* zeta / 2 with zeta the
 * orientation factor. These cross sections feed dfmi/collision.py, which forms the reduced collision
 * integrals Omega(1,1)*, Omega(2,2)*, averages them over orientations and tabulates them on Cantera's
 * MMCollisionInt grid (the tables Cantera 2.6 interpolates in GasTransport::fitProperties, which
 * wrote the reference's thermo_<mech>.txt files).
 *
 * Method (classical two-body scattering, reduced units):
 *   chi(b, E) = pi - 2 (b/r_m) int_0^1 du / sqrt(F(u)),  F(u) = 1 - (b u / r_m)^2 - V(r_m/u)/E,
 *   r_m the outermost turning point; F is evaluated in the cancellation-free form F(u) - F(1) and the
 *   integral is taken in y = -ln(1-u) by adaptive Gauss-Kronrod (7/15), split at the centrifugal barrier
 *   when the trajectory passes just over it.
 *   Q(l)(E) = 2 pi int_0^inf (1 - cos^l chi) b db by panel Gauss-Legendre, the panels clustered
 *   geometrically on both sides of the orbiting impact parameter b_o(E) (E below the orbiting energy),
 *   where chi diverges logarithmically.
 *   Q(l)* = Q(l) / (pi [1 - (1 + (-1)^l) / (2 (1 + l))])  (rigid-sphere normalisation).
 *
 * Usage: collision_q <d_min> <d_max> <n_d> <E_min> <E_max> <n_E>  -> stdout lines "d E Q1* Q2*".
 * Build: gcc -O2 -fopenmp -o collision_q collision_q.c -lm  (scripts/gen_collision_tables.py).
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

static double pot(double r, double d) {
  double i3 = 1.0 / (r * r * r), i6 = i3 * i3;
  return 4.0 * (i6 * i6 - i6 - d * i3);
}
static double dpot(double r, double d) {   /* dV/dr */
  double i = 1.0 / r, i3 = i * i * i, i6 = i3 * i3;
  return 4.0 * (-12.0 * i6 * i6 * i + 6.0 * i6 * i + 3.0 * d * i3 * i);
}
/* orbiting energy at barrier radius r: E_o = V + r V'/2 */
static double e_orb(double r, double d) {
  double i3 = 1.0 / (r * r * r), i6 = i3 * i3;
  return -20.0 * i6 * i6 + 8.0 * i6 + 2.0 * d * i3;
}

typedef struct { double E, b, rm, d, beta2, c12, c6, c3; } Traj;

/* F(w) with w = 1 - u, written as F(u) - F(1) so that it stays accurate as w -> 0 */
static double Fw(const Traj* t, double w) {
  double e12, e6, e3;
  if (w < 1e-3) {
    double l = log1p(-w);
    e12 = expm1(12.0 * l); e6 = expm1(6.0 * l); e3 = expm1(3.0 * l);
  } else {
    double u = 1.0 - w, u3 = u * u * u, u6 = u3 * u3;
    e12 = u6 * u6 - 1.0; e6 = u6 - 1.0; e3 = u3 - 1.0;
  }
  return t->beta2 * w * (2.0 - w) - (4.0 / t->E) * (t->c12 * e12 - t->c6 * e6 - t->d * t->c3 * e3);
}
static double integrand(const Traj* t, double y) {
  double w = exp(-y);
  double f = Fw(t, w);
  if (!(f > 0.0)) return 0.0;
  return w / sqrt(f);
}

static const double XGK[8] = {0.991455371120812639206854697526329, 0.949107912342758524526189684047851,
                              0.864864423359769072789712788640926, 0.741531185599394439863864773280788,
                              0.586087235467691130294144845693013, 0.405845151377397166906606412076961,
                              0.207784955007898467600689403773245, 0.000000000000000000000000000000000};
static const double WGK[8] = {0.022935322010529224963732008058970, 0.063092092629978553290700663189204,
                              0.104790010322250183839876322541518, 0.140653259715525918745189590510238,
                              0.169004726639267902826583426598550, 0.190350578064785409913256402421014,
                              0.204432940075298892414161999234649, 0.209482141084727828012999174891714};
static const double WG[4] = {0.129484966168869693270611432679082, 0.279705391489276667901467771423780,
                             0.381830050505118944950369775488975, 0.417959183673469387755102040816327};

static double gk15(const Traj* t, double a, double b, double* err) {
  double c = 0.5 * (a + b), h = 0.5 * (b - a);
  double fc = integrand(t, c);
  double rk = fc * WGK[7], rg = fc * WG[3];
  for (int j = 0; j < 7; j++) {
    double x = h * XGK[j];
    double f = integrand(t, c - x) + integrand(t, c + x);
    rk += WGK[j] * f;
    if (j & 1) rg += WG[j / 2] * f;
  }
  *err = fabs((rk - rg) * h);
  return rk * h;
}
/* globally adaptive Gauss-Kronrod over the given break points: the interval with the largest error
 * estimate is halved until the summed estimate meets tol or MAXI intervals exist (a bounded budget: next
 * to an orbiting barrier F is only known to ~1e-14 absolute, so no tolerance is reachable there) */
#define MAXI 400
static double integrate(const Traj* t, const double* brk, int nbrk, double tol) {
  double A[MAXI], B[MAXI], R[MAXI], Er[MAXI];
  int n = 0;
  double tot = 0.0, terr = 0.0;
  for (int k = 0; k + 1 < nbrk; k++) {
    A[n] = brk[k]; B[n] = brk[k + 1];
    R[n] = gk15(t, A[n], B[n], &Er[n]);
    tot += R[n]; terr += Er[n]; n++;
  }
  while (terr > tol + 1e-13 * fabs(tot) && n < MAXI) {
    int w = 0;
    for (int k = 1; k < n; k++) if (Er[k] > Er[w]) w = k;
    double a = A[w], b = B[w], m = 0.5 * (a + b);
    double e1, e2;
    double r1 = gk15(t, a, m, &e1), r2 = gk15(t, m, b, &e2);
    tot += r1 + r2 - R[w]; terr += e1 + e2 - Er[w];
    B[w] = m; R[w] = r1; Er[w] = e1;
    A[n] = m; B[n] = b; R[n] = r2; Er[n] = e2; n++;
  }
  return tot;
}

/* outermost turning point: scan F(r) = 1 - b^2/r^2 - V/E downward on a log grid (plus the orbiting
 * radius r_o, where F < 0 whenever b > b_o), bisect the first sign change */
static double turning_point(double E, double b, double d, double r_o) {
  double rhi = fmax(2.0 * b, fmax(3.0, 2.0 * cbrt(32.0 * (1.0 + fabs(d)) / E)));
  const int N = 400;
  double rlo = 0.25;
  double q = pow(rlo / rhi, 1.0 / N);
  double rprev = rhi, r = rhi;
  int found = 0;
  int ro_used = (r_o <= 0.0);
  for (int k = 1; k <= N + 1; k++) {
    double rn = rhi * pow(q, k);
    if (!ro_used && rn <= r_o) { rn = r_o; ro_used = 1; k--; }
    double f = 1.0 - b * b / (rn * rn) - pot(rn, d) / E;
    if (f < 0.0) { r = rn; found = 1; break; }
    rprev = rn;
  }
  if (!found) { fprintf(stderr, "no turning point E=%g b=%g d=%g\n", E, b, d); exit(2); }
  double lo = r, hi = rprev;       /* F(lo) < 0 <= F(hi) */
  for (int it = 0; it < 200 && hi - lo > 1e-15 * hi; it++) {
    double m = 0.5 * (lo + hi);
    double f = 1.0 - b * b / (m * m) - pot(m, d) / E;
    if (f < 0.0) lo = m; else hi = m;
  }
  return hi;
}

static double deflection(double E, double b, double d, double r_o) {
  if (b == 0.0) return M_PI;
  Traj t;
  t.E = E; t.b = b; t.d = d;
  t.rm = turning_point(E, b, d, r_o);
  double i3 = 1.0 / (t.rm * t.rm * t.rm);
  t.c3 = i3; t.c6 = i3 * i3; t.c12 = t.c6 * t.c6;
  t.beta2 = (b / t.rm) * (b / t.rm);
  /* barrier just passed over: F has a small interior minimum; split the y integral there */
  double ysplit = -1.0;
  {
    double best = 1e300, wb = 0.0;
    for (int k = 1; k < 64; k++) {
      double w = (double)k / 64.0;
      double f = Fw(&t, w);
      if (f < best) { best = f; wb = w; }
    }
    if (best < 0.2) {
      double lo = fmax(wb - 1.0 / 64.0, 1e-12), hi = fmin(wb + 1.0 / 64.0, 1.0 - 1e-12);
      for (int it = 0; it < 100; it++) {     /* golden section on F(w) */
        double m1 = hi - 0.6180339887498949 * (hi - lo), m2 = lo + 0.6180339887498949 * (hi - lo);
        if (Fw(&t, m1) < Fw(&t, m2)) hi = m2; else lo = m1;
      }
      ysplit = -log(0.5 * (lo + hi));
    }
  }
  double brk[12] = {0.0, 0.5, 1.5, 3.0, 6.0, 12.0, 24.0, 48.0, 96.0, 200.0};
  int nbrk = 10;
  if (ysplit > 0.0 && ysplit < 200.0) {        /* insert the barrier position as a break point */
    int k = nbrk;
    while (k > 0 && brk[k - 1] > ysplit) { brk[k] = brk[k - 1]; k--; }
    brk[k] = ysplit; nbrk++;
  }
  double I = integrate(&t, brk, nbrk, 1e-12);
  return M_PI - 2.0 * sqrt(t.beta2) * I;
}

/* 16-point Gauss-Legendre on [-1, 1] */
static const double GLX[8] = {0.0950125098376374, 0.2816035507792589, 0.4580167776572274, 0.6178762444026438,
                              0.7554044083550030, 0.8656312023878318, 0.9445750230732326, 0.9894009349916499};
static const double GLW[8] = {0.1894506104550685, 0.1826034150449236, 0.1691565193950025, 0.1495959888165767,
                              0.1246289712555339, 0.0951585116824928, 0.0622535239386479, 0.0271524594117541};

static void panel(double E, double d, double r_o, double a, double c, double* q1, double* q2) {
  double m = 0.5 * (a + c), h = 0.5 * (c - a);
  for (int j = 0; j < 8; j++) {
    for (int s = -1; s <= 1; s += 2) {
      double b = m + s * h * GLX[j];
      double chi = deflection(E, b, d, r_o);
      double cc = cos(chi);
      *q1 += GLW[j] * h * (1.0 - cc) * b;
      *q2 += GLW[j] * h * (1.0 - cc * cc) * b;
    }
  }
}

/* orbiting parameters for energy E: returns b_o (0 if none) and the barrier radius r_o */
static double orbit(double E, double d, double* r_o) {
  /* E_o(r) on the outer side of its maximum */
  double rmax = 1.0, emax = -1e300;
  for (int k = 0; k <= 4000; k++) {
    double r = 0.8 * pow(200.0 / 0.8, k / 4000.0);
    double e = e_orb(r, d);
    if (e > emax) { emax = e; rmax = r; }
  }
  *r_o = 0.0;
  if (!(E < emax)) return 0.0;
  /* bracket the outer root of E_o(r) = E beyond rmax (E_o decreasing there) */
  double lo = rmax, hi = rmax;
  while (e_orb(hi, d) > E) { hi *= 1.5; if (hi > 1e6) return 0.0; }
  for (int it = 0; it < 200; it++) {
    double m = 0.5 * (lo + hi);
    if (e_orb(m, d) > E) lo = m; else hi = m;
  }
  double r = 0.5 * (lo + hi);
  double L = r * r * r * dpot(r, d) / 2.0;   /* E b^2 */
  if (!(L > 0.0)) return 0.0;
  *r_o = r;
  return sqrt(L / E);
}

int main(int argc, char** argv) {
  if (argc != 7) {
    fprintf(stderr, "usage: collision_q d_min d_max n_d E_min E_max n_E\n");
    return 1;
  }
  double dmin = atof(argv[1]), dmax = atof(argv[2]);
  int nd = atoi(argv[3]);
  double emin = atof(argv[4]), emax = atof(argv[5]);
  int nE = atoi(argv[6]);
  int n = nd * nE;
  double* out = (double*)calloc((size_t)n * 4, sizeof(double));
#pragma omp parallel for schedule(dynamic, 1)
  for (int idx = 0; idx < n; idx++) {
    int id = idx / nE, ie = idx % nE;
    double d = nd > 1 ? dmin + (dmax - dmin) * id / (nd - 1) : dmin;
    double E = nE > 1 ? emin * pow(emax / emin, (double)ie / (nE - 1)) : emin;
    double r_o;
    double bo = orbit(E, d, &r_o);
    double bmax = fmax(8.0, 20.0 * cbrt(4.0 * (1.0 + fabs(d)) / E));
    double q1 = 0.0, q2 = 0.0;
    /* panel edges: geometric in b, with dense clustering around b_o */
    double bs[1024];
    int nb = 0;
    bs[nb++] = 0.0;
    double b = 0.05;
    while (b < bmax) { bs[nb++] = b; b *= 1.03; }
    bs[nb++] = bmax;
    if (bo > 0.0 && bo < bmax) {
      /* replace the edges within a factor 1.5 of b_o by clustered ones */
      double tmp[1024];
      int nt = 0;
      for (int k = 0; k < nb; k++)
        if (bs[k] < bo / 1.5 || bs[k] > bo * 1.5) tmp[nt++] = bs[k];
      double cl[200];
      int nc = 0;
      for (int k = 1; k <= 48; k++) cl[nc++] = bo * (1.0 - pow(2.0, -k) * (1.0 / 3.0) * 2.0);
      for (int k = 48; k >= 1; k--) cl[nc++] = bo * (1.0 + pow(2.0, -k));
      /* merge */
      int i = 0, j = 0, m = 0;
      double merged[1280];
      while (i < nt || j < nc) {
        if (j >= nc || (i < nt && tmp[i] < cl[j])) merged[m++] = tmp[i++];
        else merged[m++] = cl[j++];
      }
      nb = 0;
      for (int k = 0; k < m; k++) bs[nb++] = merged[k];
      /* interval [b_o (1 - 2^-48 ...), b_o (1 + 2^-48)] is left out: its measure is < 1e-14 b_o */
      for (int k = 0; k + 1 < nb; k++) {
        if (bs[k] < bo && bs[k + 1] > bo) continue;
        panel(E, d, r_o, bs[k], bs[k + 1], &q1, &q2);
      }
    } else {
      for (int k = 0; k + 1 < nb; k++) panel(E, d, r_o, bs[k], bs[k + 1], &q1, &q2);
    }
    /* Q(l) = 2 pi int (...) b db;  Q* = Q / (pi * norm_l), norm_1 = 1, norm_2 = 2/3 */
    out[4 * idx + 0] = d;
    out[4 * idx + 1] = E;
    out[4 * idx + 2] = 2.0 * q1;
    out[4 * idx + 3] = 2.0 * q2 / (2.0 / 3.0);
  }
  for (int idx = 0; idx < n; idx++)
    printf("%.10f %.17g %.17g %.17g\n", out[4 * idx], out[4 * idx + 1], out[4 * idx + 2], out[4 * idx + 3]);
  free(out);
  return 0;
}
