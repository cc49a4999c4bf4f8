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


def hf298_per_mass(nasa, W):
    """hc_i = Hf298SS_i / W_i [J/kg], dfChemistryModel.C:335-338. Cantera's NasaPoly2::reportHf298 takes the
    NASA7 range holding 298.15 K (the low range when 298.15 <= T_mid) and NasaPoly1::updateProperties'
    h/RT = ct0 + ct1/2 + ct2/3 + ct3/4 + ct4/5 + a5/T with ct_k = a_k T^k, times GasConstant * 298.15; the same
    expression in the same order as the library's heat_of_formation_per_mass (thermo.hip), scalar Python floats."""
    T = 298.15
    T2 = T * T
    T3 = T2 * T
    T4 = T3 * T
    rT = 1.0 / T
    out = np.zeros(len(W))
    for i, row in enumerate(np.asarray(nasa, dtype=np.float64)):
        a = [float(v) for v in (row[8:15] if T <= row[0] else row[1:8])]
        ct0, ct1, ct2, ct3, ct4 = a[0], a[1] * T, a[2] * T2, a[3] * T3, a[4] * T4
        h_RT = ct0 + 0.5 * ct1 + (1.0 / 3.0) * ct2 + 0.25 * ct3 + 0.2 * ct4 + a[5] * rT
        out[i] = h_RT * RU * T / float(W[i])
    return out


def heat_release(hc, RR):
    """Qdot per cell = -sum_i hc_i RR_i, accumulated species by species from 0 (dfChemistryModel.C:753,771;
    the DF-ODENet path pytorchFunctions.H:233-238). RR [S, n] -> Qdot [n]."""
    RR = np.asarray(RR, dtype=np.float64)
    q = np.zeros(RR.shape[1])
    for i in range(RR.shape[0]):
        q = q - float(hc[i]) * RR[i]
    return q


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

    def heat_release(self, RR):
        """Qdot = -sum_i hc_i RR_i of reaction rates RR [S, n] (dfChemistryModel.C:771)."""
        return heat_release(hf298_per_mass(self.nasa, self.W), RR)

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
