"""CPU oracle for the per-cell stiff chemistry (TEST INFRASTRUCTURE -- never the product path).

Restates the reference's chemistry semantics, dfChemistryModel::solveSingle
(src/dfChemistryModel/dfChemistryModel.C:737-780): each cell is integrated over the time step as a
closed, constant-volume reactor at FIXED temperature and density (Cantera Reactor with the energy
equation disabled), and the source term is RR_i = (Y_i(dt) - Y_i(0)) * rho / dt.
Reaction rates follow Cantera 2.6 GasKinetics (the third-party dependency named in SURVEY.md 8c,
libcantera-devel 2.6, absent here): Arrhenius k = A T^b exp(-Ta/T); three-body [M] = sum eff_i C_i;
Lindemann / Troe fall-off; reverse rates from NASA7 equilibrium constants,
Kc = exp(-dG0/RT) (p_atm / RT)^dnu. Integration: SciPy BDF with tight tolerances.

Parity status: the kinetics/integration are NOT pinned to Cantera (no Cantera here and no reference
test pins chemistry outputs -- "parity unpinned"); tests check invariants (element
conservation, detailed balance, equilibrium limit) and the GPU integrator against this oracle.
"""
from __future__ import annotations

import numpy as np
from scipy.integrate import solve_ivp

RU = 8314.46261815324   # J/kmol/K
P_ATM = 101325.0


def g_RT(nasa, T):
    """Gibbs free energy / RT per species from NASA7 rows [Tmid, hi a0..a6, lo a0..a6]."""
    out = np.zeros(nasa.shape[0])
    for i, row in enumerate(nasa):
        a = row[1:8] if T > row[0] else row[8:15]
        h = a[0] + a[1] * T / 2 + a[2] * T ** 2 / 3 + a[3] * T ** 3 / 4 + a[4] * T ** 4 / 5 + a[5] / T
        s = a[0] * np.log(T) + a[1] * T + a[2] * T ** 2 / 2 + a[3] * T ** 3 / 3 + a[4] * T ** 4 / 4 + a[6]
        out[i] = h - s
    return out


class Kinetics:
    def __init__(self, mech, nasa, W):
        self.m = mech
        self.nasa = np.asarray(nasa)
        self.W = np.asarray(W)

    def rate_constants(self, T):
        m = self.m
        kf = m.A * T ** m.b * np.exp(-m.Ta / T)
        k0 = m.A0 * T ** m.b0 * np.exp(-m.Ta0 / T)
        g = g_RT(self.nasa, T)
        dG = np.zeros(m.R); dnu = np.zeros(m.R)
        for r in range(m.R):
            for k in range(3):
                if m.prod[r, k] >= 0:
                    dG[r] += m.nu_p[r, k] * g[m.prod[r, k]]; dnu[r] += m.nu_p[r, k]
                if m.reac[r, k] >= 0:
                    dG[r] -= m.nu_r[r, k] * g[m.reac[r, k]]; dnu[r] -= m.nu_r[r, k]
        Kc = np.exp(-dG) * (P_ATM / (RU * T)) ** dnu
        return kf, k0, Kc

    def rates_of_progress(self, T, C, consts=None):
        m = self.m
        kf, k0, Kc = consts if consts is not None else self.rate_constants(T)
        q = np.zeros(m.R)
        for r in range(m.R):
            k = kf[r]
            M = float(np.dot(m.eff[r], C)) if m.itype[r] != 0 else 1.0
            if m.itype[r] >= 2:
                Pr = k0[r] * M / kf[r]
                F = 1.0
                if m.itype[r] == 3:
                    A, T3, T1, T2 = m.troe[r]
                    Fc = (1 - A) * np.exp(-T / T3) + A * np.exp(-T / T1) + (np.exp(-T2 / T) if m.has_T2[r] else 0.0)
                    lFc = np.log10(max(Fc, 1e-300))
                    c = -0.4 - 0.67 * lFc
                    n = 0.75 - 1.27 * lFc
                    lPr = np.log10(max(Pr, 1e-300))
                    f1 = (lPr + c) / (n - 0.14 * (lPr + c))
                    F = 10.0 ** (lFc / (1 + f1 * f1))
                k = kf[r] * Pr / (1 + Pr) * F
                M = 1.0
            fwd = k
            for j in range(3):
                if m.reac[r, j] >= 0:
                    fwd *= C[m.reac[r, j]] ** m.nu_r[r, j]
            rev = 0.0
            if m.reversible[r]:
                rev = k / Kc[r]
                for j in range(3):
                    if m.prod[r, j] >= 0:
                        rev *= C[m.prod[r, j]] ** m.nu_p[r, j]
            q[r] = M * (fwd - rev)
        return q

    def production_rates(self, T, C, consts=None):
        m = self.m
        q = self.rates_of_progress(T, C, consts)
        w = np.zeros(m.S)
        for r in range(m.R):
            for j in range(3):
                if m.reac[r, j] >= 0:
                    w[m.reac[r, j]] -= m.nu_r[r, j] * q[r]
                if m.prod[r, j] >= 0:
                    w[m.prod[r, j]] += m.nu_p[r, j] * q[r]
        return w

    def reactor_state(self, T, p, Y):
        """Cantera setState_TPY(T, p, Y) (dfChemistryModel.C:755): Phase::setMassFractions clips at 0 and
        normalises; density = p * meanW / (R T). Returns (density, normalised Y)."""
        y = np.maximum(np.asarray(Y, dtype=np.float64), 0.0)
        y = y / y.sum()
        return p / ((y / self.W).sum() * RU * T), y

    def integrate_cell(self, T, rho, Y, dt, rtol=1e-11, atol=1e-22):
        """Closed constant-volume reactor at fixed T and density rho over dt -> Y(dt)."""
        C0 = rho * np.asarray(Y) / self.W
        consts = self.rate_constants(T)
        f = lambda t, C: self.production_rates(T, C, consts)
        sol = solve_ivp(f, (0.0, dt), C0, method="BDF", rtol=rtol, atol=atol)
        if not sol.success:
            raise RuntimeError(sol.message)
        return sol.y[:, -1] * self.W / rho

    def reaction_rates(self, T, p, rho, Y, dt, **kw):
        """RR [S, n] = (Y(dt) - Y) rho / dt for each cell (columns of Y), dfChemistryModel::solveSingle
        (:737-780): the reactor state is setState_TPY(T, p, Y); `rho` is the thermo density the
        difference is scaled by (problem.rhoi = rho_[celli], :807). p = None: the reactor runs at `rho`."""
        Y = np.asarray(Y)
        out = np.zeros_like(Y)
        for c in range(Y.shape[1]):
            if p is None:
                rc, y0 = float(rho[c]), Y[:, c]
            else:
                rc, y0 = self.reactor_state(float(T[c]), float(p[c]), Y[:, c])
            Yn = self.integrate_cell(float(T[c]), rc, y0, dt, **kw)
            out[:, c] = (Yn - Y[:, c]) * rho[c] / dt
        return out
