#!/usr/bin/env python3
"""does a Rosenbrock-W method with a reused Jacobian do less chemistry work per flow step than
the production ROS3 (chem.hip k_chem_gen: one analytic Jacobian + LU per step, three stages, two rate evaluations)?

Prototype on the CPU (numpy, FD Jacobians), on cells of the headline's own state (tests/golden/tgv64, Burke 2012,
rtol 1e-6 / atol 1e-10, dt 1e-6 s, two consecutive flow steps, the second starting from the first's last step size as
the kernel does). Integrators, all with the kernel's error norm and step-size controller:
  ros3        the production scheme (KPP ROS3 constants of chem.hip), fresh Jacobian every step
  ros34pw2    Rang & Angermann's W-method (4 stages, order 3, W-order 2), fresh Jacobian every step
  ros34pw2-J  the same with ONE Jacobian per cell and flow step (refreshed after a rejected step), LU per step
  ros3-J      ROS3 with the frozen Jacobian (not a W-method: shows what the order conditions buy)
Cost per cell = sum over its steps of the generated kernel's VALU instructions per component, counted from the gfx950
ISA of one-function probe kernels over chem_gen_burke9.inc (wdot, wdot+Jacobian, LU factor, LU solve; the counts
are the arguments below). Accuracy: max over the sampled cells of |RR - RR_BDF| / species scale (RR_BDF: SciPy BDF,
rtol 1e-10). Output -> stdout (profiles/r06_chem_w_proto.txt).
"""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "deepflame-dev_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from chem_oracle import Kinetics   # noqa: E402
from dfmi.kinetics import parse_mechanism           # noqa: E402
from dfmi.mech import read_yaml_mechanism           # noqa: E402
from dfmi.foam_io import read_case_fields           # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")
# VALU instructions per call on gfx950 (probe kernels over chem_gen_burke9.inc, the probe's own loads/stores
# subtracted): rates only, rates + dense analytic Jacobian, LU factor of the 8x8 active block, one LU solve;
# STAGE = the per-stage vector work (stage point, right-hand side, error-norm share), measured from k_chem_gen
COST = dict(wdot=480, jac=900, lu=220, sol=70, stage=50)


class Rates:
    """Reaction-vectorised restatement of chem_oracle.Kinetics.production_rates (same formulas)."""

    def __init__(self, m, nasa, W):
        self.m, self.nasa, self.W = m, np.asarray(nasa), np.asarray(W)
        self.S = m.S
        self.ri = np.where(m.reac >= 0, m.reac, self.S)
        self.pi = np.where(m.prod >= 0, m.prod, self.S)
        self.nr = np.where(m.reac >= 0, m.nu_r, 0.0)
        self.np_ = np.where(m.prod >= 0, m.nu_p, 0.0)
        self.nu = np.zeros((m.R, self.S + 1))
        for r in range(m.R):
            for j in range(3):
                self.nu[r, self.ri[r, j]] -= self.nr[r, j]
                self.nu[r, self.pi[r, j]] += self.np_[r, j]
        self.nu = self.nu[:, :self.S]

    def consts(self, T):
        return Kinetics(self.m, self.nasa, self.W).rate_constants(T)

    def wdot(self, T, C, k):
        m = self.m
        kf, k0, Kc = k
        Cp = np.append(C, 1.0)
        M = m.eff @ C
        kk = kf.copy()
        third = m.itype != 0
        fo = m.itype >= 2
        Mx = np.where(third & ~fo, M, 1.0)
        if fo.any():
            Pr = k0[fo] * M[fo] / kf[fo]
            F = np.ones(Pr.size)
            tr = m.itype[fo] == 3
            if tr.any():
                A, T3, T1, T2 = (m.troe[fo][tr][:, i] for i in range(4))
                Fc = (1 - A) * np.exp(-T / T3) + A * np.exp(-T / T1) + np.where(m.has_T2[fo][tr], np.exp(-T2 / T), 0.0)
                lFc = np.log10(np.maximum(Fc, 1e-300))
                c = -0.4 - 0.67 * lFc
                n = 0.75 - 1.27 * lFc
                lPr = np.log10(np.maximum(Pr[tr], 1e-300))
                f1 = (lPr + c) / (n - 0.14 * (lPr + c))
                F[tr] = 10.0 ** (lFc / (1 + f1 * f1))
            kk[fo] = kf[fo] * Pr / (1 + Pr) * F
        fwd = kk * np.prod(Cp[self.ri] ** self.nr, axis=1)
        rev = np.where(m.reversible, kk / Kc * np.prod(Cp[self.pi] ** self.np_, axis=1), 0.0)
        return self.nu.T @ (Mx * (fwd - rev))

    def jac(self, T, C, k, f0):
        J = np.zeros((self.S, self.S))
        for j in range(self.S):
            d = 1e-7 * abs(C[j]) + 1e-22
            Cd = C.copy()
            Cd[j] += d
            J[:, j] = (self.wdot(T, Cd, k) - f0) / d
        return J


def tableau(name):
    """Transformed Rosenbrock coefficients (a, c, m, e, gamma) of (I - h gamma J) U_i = h gamma (f(y + sum a_ij U_j)
    + sum c_ij U_j / h), y+ = y + sum m_i U_i, err = sum e_i U_i."""
    if name == "ros3":   # chem.hip k_chem_gen constants (KPP ROS3)
        g = 0.43586652150845899941601945119356
        a = np.array([[0, 0, 0], [1, 0, 0], [1, 0, 0]], float)
        c = np.array([[0, 0, 0], [-0.10156171083877702091975600115545e1, 0, 0],
                      [0.40759956452537699824805835358067e1, 0.92076794298330791242156818474003e1, 0]])
        m = np.array([1.0, 0.61697947043828245592553615689730e1, -0.42772256543218573326238373806514])
        e = np.array([0.5, -0.29079558716805469821718236208017e1, 0.22354069897811569627360909276199])
        return a, c, m, e, g
    # ROS34PW2 (Rang & Angermann 2005), untransformed alpha / gamma / b / bhat
    g = 4.3586652150845900e-01
    al = np.zeros((4, 4)); ga = np.zeros((4, 4))
    al[1, 0] = 8.7173304301691801e-01
    al[2, 0], al[2, 1] = 8.4457060015369423e-01, -1.1299064236484185e-01
    al[3, 2] = 1.0
    ga[1, 0] = -8.7173304301691801e-01
    ga[2, 0], ga[2, 1] = -9.0338057013044082e-01, 5.4180672388095326e-02
    ga[3, 0], ga[3, 1], ga[3, 2] = 2.4212380706095346e-01, -1.2232505839045147e+00, 5.4526025533510214e-01
    b = np.array([2.4212380706095346e-01, -1.2232505839045147e+00, 1.5452602553351020e+00, 4.3586652150845900e-01])
    bh = np.array([3.7810903145819369e-01, -9.6042292212423178e-02, 5.0e-01, 2.1793326075422950e-01])
    G = ga + g * np.eye(4)
    Gi = np.linalg.inv(G)
    return al @ Gi, np.diag(np.full(4, 1 / g)) - Gi, b @ Gi, (b - bh) @ Gi, g


def check_order(name, J_exact=True):
    """Observed order on an autonomous nonlinear 2x2 system (h-halving); J exact or a fixed wrong matrix (W-property)."""
    a, c, m, e, g = tableau(name)
    f = lambda t, y: np.array([-y[0] ** 2 + y[1], -0.5 * y[1] + y[0]])
    Jf = lambda y: np.array([[-2 * y[0], 1.0], [1.0, -0.5]]) if J_exact else np.zeros((2, 2))
    errs = []
    for n in (20, 40, 80):
        h, y = 1.0 / n, np.array([1.0, 0.5])
        for k in range(n):
            Jm = np.eye(2) - h * g * (Jf(y) if J_exact else np.array([[-1.0, 0.3], [0.2, -0.4]]))
            U = []
            for i in range(len(m)):
                yi = y + sum(a[i, j] * U[j] for j in range(i))
                U.append(np.linalg.solve(Jm, h * g * (f(k * h, yi) + sum(c[i, j] * U[j] for j in range(i)) / h)))
            y = y + sum(m[i] * U[i] for i in range(len(m)))
        errs.append(y)
    # Richardson-style order estimate from three resolutions
    d1, d2 = np.abs(errs[0] - errs[1]).max(), np.abs(errs[1] - errs[2]).max()
    return np.log2(d1 / d2)


def integrate(rt, T, C0, dt, rho, method, hp, rtol=1e-6, atol=1e-10):
    """One flow step of one cell; returns (C, hnext, counts)."""
    name = "ros3" if method.startswith("ros3") and not method.startswith("ros34") else "ros34pw2"
    frozen = method.endswith("-J")
    a, c, m, e, g = tableau(name)
    s = len(m)
    k = rt.consts(T)
    cnt = dict(wdot=0, jac=0, lu=0, sol=0, stage=0, steps=0, rej=0)
    y = C0.copy()
    t, h = 0.0, (min(dt, hp) if hp > 0 else dt)
    J = None
    arho = atol * rho
    while t < dt:
        if cnt["steps"] + cnt["rej"] > 5000:
            raise RuntimeError("too many steps")
        if t + h > dt:
            h = dt - t
        f0 = rt.wdot(T, y, k)
        if J is None or not frozen:
            J = rt.jac(T, y, k, f0)
            cnt["jac"] += 1
        else:
            cnt["wdot"] += 1
        A = np.eye(rt.S) - h * g * J
        cnt["lu"] += 1
        U = []
        for i in range(s):
            if i == 0:
                fi = f0
            elif i == 1 or not np.array_equal(a[i, :i], np.append(a[i - 1, :i - 1], 0.0)):
                yi = y + sum(a[i, j] * U[j] for j in range(i))
                fi = rt.wdot(T, yi, k)
                cnt["wdot"] += 1
            U.append(np.linalg.solve(A, h * g * (fi + sum(c[i, j] * U[j] for j in range(i)) / h)))
            cnt["sol"] += 1
            cnt["stage"] += 1
        yn = y + sum(m[i] * U[i] for i in range(s))
        er = sum(e[i] * U[i] for i in range(s)) / (arho / rt.W + rtol * np.maximum(np.abs(y), np.abs(yn)))
        err = np.sqrt((er * er).sum() / rt.S)
        if err <= 1.0:
            y, t = yn, t + h
            cnt["steps"] += 1
            fac = 0.9 * err ** (-1 / 3) if err > 0 else 5.0
            h *= min(5.0, max(0.2, fac))
        else:
            cnt["rej"] += 1
            h *= min(0.5, max(0.1, 0.9 * err ** (-1 / 3)))
            if frozen:
                J = None   # a rejected step refreshes the Jacobian
    return y, h, cnt


def main():
    ym = read_yaml_mechanism(os.path.join(GOLDEN, "Burke2012_s9r23.yaml"))
    mech = parse_mechanism(os.path.join(GOLDEN, "Burke2012_s9r23.yaml"))
    rt = Rates(mech, ym["nasa"], ym["W"])
    kin = Kinetics(mech, ym["nasa"], ym["W"])
    src = read_case_fields(os.path.join(GOLDEN, "tgv64"), ym["species"])
    for nm in ("ros3", "ros34pw2"):
        print(f"# observed order {nm}: exact J {check_order(nm):.2f}, fixed wrong J {check_order(nm, False):.2f}")
    rng = np.random.default_rng(6)
    n = int(os.environ.get("NCELLS", "400"))
    Ts = src["T"]
    # half uniform over the box, half from the hottest 5 % (where the integration steps are)
    hot = np.argsort(Ts)[-len(Ts) // 20:]
    sel = np.concatenate([rng.choice(len(Ts), n // 2, replace=False), rng.choice(hot, n - n // 2, replace=False)])
    dt = 1e-6
    methods = ["ros3", "ros34pw2", "ros34pw2-J", "ros3-J"]
    print(f"# {n} cells of tests/golden/tgv64 ({n // 2} uniform, {n - n // 2} from the hottest 5 %), dt {dt}, "
          f"rtol 1e-6 atol 1e-10; per-call VALU instruction costs {COST}")
    tot = {mt: {k: 0 for k in ("wdot", "jac", "lu", "sol", "stage", "steps", "rej")} for mt in methods}
    err = {mt: 0.0 for mt in methods}
    RRs = {mt: [] for mt in methods}
    ref = []
    for ci in sel:
        T, p = float(Ts[ci]), float(src["p"][ci])
        rho, y0 = kin.reactor_state(T, p, src["Y"][:, ci])
        C0 = rho * y0 / rt.W
        # flow step 1 (seeds the step size), then flow step 2 from its result: the steady solve the bench times
        C1, h1, _ = integrate(rt, T, C0, dt, rho, "ros3", 0.0)
        for mt in methods:
            C2, _, cn = integrate(rt, T, C1, dt, rho, mt, h1)
            for k_ in cn:
                tot[mt][k_] += cn[k_]
            RRs[mt].append((C2 * rt.W / rho - C1 * rt.W / rho) * rho / dt)
        Yr = kin.integrate_cell(T, rho, C1 * rt.W / rho, dt, rtol=1e-10, atol=1e-20)
        ref.append((Yr - C1 * rt.W / rho) * rho / dt)
    ref = np.array(ref).T
    scale = np.maximum(np.abs(ref).max(axis=1, keepdims=True), 1e-3 * np.abs(ref).max())
    print(f"{'method':12s} {'steps':>7s} {'rej':>5s} {'jac':>6s} {'wdot':>6s} {'lu':>6s} {'solve':>6s} "
          f"{'VALU/cell':>10s} {'vs ros3':>8s} {'max RR err':>11s}")
    base = None
    for mt in methods:
        c = tot[mt]
        cost = sum(COST[k] * c[k] for k in ("wdot", "jac", "lu", "sol", "stage")) / n
        base = base or cost
        e = (np.abs(np.array(RRs[mt]).T - ref) / scale).max()
        print(f"{mt:12s} {c['steps'] / n:7.2f} {c['rej'] / n:5.2f} {c['jac'] / n:6.2f} {c['wdot'] / n:6.2f} "
              f"{c['lu'] / n:6.2f} {c['sol'] / n:6.2f} {cost:10.0f} {cost / base:8.3f} {e:11.2e}")


if __name__ == "__main__":
    main()
