"""Transport-property fits for the GPU thermo table.

Writes ``thermo_<mech>.txt`` (format: dfmi.mech / reference src_gpu/dfThermo.cu:361-435) from a
Cantera YAML mechanism, restating Cantera 2.6 ``GasTransport::fitProperties`` (mixture-averaged,
polynomial degree 4 in ln T, 50 points between the phase's minTemp and maxTemp, relative
least-squares weights):
  * pure-species viscosity, Chapman-Enskog:  mu = 5/16 sqrt(pi m k T) / (pi sigma^2 Omega22*)
    fitted as sqrt(mu / sqrt(T));
  * conductivity, Warnatz/Kee rotational-relaxation model (Kee, Coltrin & Glarborg 2003 eq. 12.112):
    fitted as lambda / sqrt(T);
  * binary diffusion D_jk * p = 3/16 sqrt(2 pi / m_jk) (k T)^1.5 / (pi sigma_jk^2 Omega11*), fitted as
    D_jk p / T^1.5.
Combining rules and the polar/non-polar correction follow Cantera's GasTransport::setupCollision-
Parameters / makePolarCorrections.

Collision integrals: Omega22* and Omega11* = Omega22*/A* at (T*, delta*) by Cantera's MMCollisionInt
interpolation (dfmi/collision.py) of Monchick-Mason-style Stockmayer tables recomputed from the potential
(scripts/gen_collision_tables.py). Against the reference's shipped table for ES80_H2-7-16 (generated with
Cantera) the evaluated properties agree to the tolerances in tests/test_transport_fit.py: non-polar
viscosities to 1e-4, conductivities and diffusivities to 1e-3 (2.5e-3 for H2 pairs at T* > 75, where the
published Omega11* is not known), the strongly polar H2O to 1e-2 (the orientation-averaged integrals
differ from Monchick & Mason's 1961 numbers by up to 0.8 %).
"""
from __future__ import annotations

import sys
import numpy as np

from .mech import ThermoTable, read_yaml_mechanism, write_thermo_table

KB = 1.380649e-23            # J/K
NA = 6.02214076e26           # 1/kmol (Cantera units)
R = 8314.46261815324         # J/kmol/K
EPS0 = 8.8541878128e-12      # F/m
LIGHT = 299792458.0
DEBYE = 1e-21 / LIGHT        # C m
PI = np.pi


_MM = None


def _mm():
    global _MM
    if _MM is None:
        from .collision import MMCollisionInt
        _MM = MMCollisionInt()
    return _MM


def omega11(ts, delta=0.0):
    f = _mm().omega11
    return np.array([f(float(t), float(delta)) for t in np.ravel(ts)]).reshape(np.shape(ts)) if np.ndim(ts) else f(ts, delta)


def omega22(ts, delta=0.0):
    f = _mm().omega22
    return np.array([f(float(t), float(delta)) for t in np.ravel(ts)]).reshape(np.shape(ts)) if np.ndim(ts) else f(ts, delta)


def _cp_R(nasa_row, T):
    a = nasa_row[1:8] if T > nasa_row[0] else nasa_row[8:15]
    return a[0] + a[1] * T + a[2] * T ** 2 + a[3] * T ** 3 + a[4] * T ** 4


def _polyfit_rel(x, y, deg=4):
    c = np.polynomial.polynomial.polyfit(x, y, deg, w=1.0 / np.abs(y))
    return c


def fit_mechanism(ym: dict) -> ThermoTable:
    sp = ym["species"]
    S = len(sp)
    W = np.asarray(ym["W"], dtype=np.float64)
    nasa = np.asarray(ym["nasa"], dtype=np.float64)
    tr = ym["transport"]
    geom = [t.get("geometry", "atom") for t in tr]
    eps = np.array([float(t.get("well-depth", 0.0)) for t in tr]) * KB              # J
    sig = np.array([float(t.get("diameter", 0.0)) for t in tr]) * 1e-10             # m
    dip = np.array([float(t.get("dipole", 0.0)) for t in tr]) * DEBYE               # C m
    pol = np.array([float(t.get("polarizability", 0.0)) for t in tr]) * 1e-30       # m^3
    zrot = np.array([float(t.get("rotational-relaxation", 0.0)) for t in tr])
    crot = np.array([{"atom": 0.0, "linear": 1.0, "nonlinear": 1.5}[g] for g in geom])
    polar = dip > 0
    tmin = max(r[0] for r in ym["trange"])
    tmax = min(r[1] for r in ym["trange"])
    npts = 50
    T = tmin + (tmax - tmin) / (npts - 1) * np.arange(npts)
    lnT = np.log(T)

    # pair parameters (GasTransport::setupCollisionParameters)
    mred = np.outer(W, W) / (NA * (W[:, None] + W[None, :]))                        # kg
    epsij = np.sqrt(np.outer(eps, eps))
    diam = 0.5 * (sig[:, None] + sig[None, :])
    dipij = np.sqrt(np.outer(dip, dip))
    delta = 0.5 * dipij ** 2 / (4 * PI * EPS0 * epsij * diam ** 3)
    for i in range(S):
        for j in range(S):
            if polar[i] != polar[j]:               # makePolarCorrections
                kp, knp = (i, j) if polar[i] else (j, i)
                d3np, d3p = sig[knp] ** 3, sig[kp] ** 3
                alpha_star = pol[knp] / d3np
                mu_p_star = dip[kp] / np.sqrt(4 * PI * EPS0 * d3p * eps[kp])
                xi = 1.0 + 0.25 * alpha_star * mu_p_star ** 2 * np.sqrt(eps[kp] / eps[knp])
                diam[i, j] *= xi ** (-1.0 / 6.0)
                epsij[i, j] *= xi * xi
                delta[i, j] = 0.0

    visc = np.zeros((S, 5)); cond = np.zeros((S, 5)); bdiff = np.zeros((S, S, 5))
    for k in range(S):
        ts298 = KB * 298.0 / eps[k]
        fz298 = 1.0 + PI ** 1.5 / np.sqrt(ts298) * (0.5 + 1.0 / ts298) + (0.25 * PI * PI + 2) / ts298
        spv, spc = np.zeros(npts), np.zeros(npts)
        for n, t in enumerate(T):
            ts = KB * t / eps[k]
            om22 = omega22(ts, delta[k, k])
            om11 = omega11(ts, delta[k, k])
            dself = 3.0 / 16.0 * np.sqrt(2 * PI / mred[k, k]) * (KB * t) ** 1.5 / (PI * sig[k] ** 2 * om11)
            mu = 5.0 / 16.0 * np.sqrt(PI * W[k] * KB * t / NA) / (om22 * PI * sig[k] ** 2)
            f_int = W[k] / (R * t) * dself / mu
            A = 2.5 - f_int
            fz = 1.0 + PI ** 1.5 / np.sqrt(ts) * (0.5 + 1.0 / ts) + (0.25 * PI * PI + 2) / ts
            Bf = zrot[k] * fz298 / fz + 2.0 / PI * (5.0 / 3.0 * crot[k] + f_int)
            c1 = 2.0 / PI * A / Bf
            cv_int = _cp_R(nasa[k], t) - 2.5 - crot[k]
            f_rot = f_int * (1.0 + c1)
            f_trans = 2.5 * (1.0 - c1 * crot[k] / 1.5)
            lam = (mu / W[k]) * R * (f_trans * 1.5 + f_rot * crot[k] + f_int * cv_int)
            spv[n] = np.sqrt(mu / np.sqrt(t))
            spc[n] = lam / np.sqrt(t)
        visc[k] = _polyfit_rel(lnT, spv)
        cond[k] = _polyfit_rel(lnT, spc)
    for k in range(S):
        for j in range(k, S):
            ts = KB * T / epsij[j, k]
            d = 3.0 / 16.0 * np.sqrt(2 * PI / mred[k, j]) * (KB * T) ** 1.5 / (PI * diam[j, k] ** 2 *
                                                                                 omega11(ts, delta[j, k]))
            c = _polyfit_rel(lnT, d / T ** 1.5)
            bdiff[k, j] = c; bdiff[j, k] = c
    return ThermoTable(list(sp), W, nasa, visc, cond, bdiff)


def main(argv):
    if len(argv) != 2:
        print("usage: python -m dfmi.transport_fit mech.yaml thermo_out.txt")
        return 2
    t = fit_mechanism(read_yaml_mechanism(argv[0]))
    write_thermo_table(argv[1], t)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
