"""Mechanism -> HIP code generator for the chemistry fast path (chem.hip).

For a given mechanism it emits a struct with straight-line device functions -- rate constants,
production rates, analytic Jacobian, and a symbolically-sparse LU of I - h*g*J over the active species
(those with a net stoichiometric change; third-body-only species ride along as constants) -- with every species
and reaction index a compile-time constant, so the ROS3 integrator keeps the whole cell state in
registers (no LDS, no dynamic indexing). The generic, data-driven kernel in chem.hip stays the
fallback for mechanisms that were not compiled in. A fingerprint (FNV-1a over the packed mechanism
arrays, NASA7 rows and molecular weights) selects the generated code at run time only when the
uploaded mechanism is bitwise the one it was generated from.

    python -m dfmi.chem_codegen mech.yaml name out.inc
"""
from __future__ import annotations

import math
import struct
import sys

import numpy as np

from .kinetics import parse_mechanism
from .mech import read_yaml_mechanism

RU = 8314.46261815324
P_ATM = 101325.0


def fnv1a64(chunks) -> int:
    h = 0xcbf29ce484222325
    for b in chunks:
        for byte in b:
            h ^= byte
            h = (h * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return h


def fingerprint(mech, nasa, W) -> int:
    idata, irs, dd = mech.pack()
    return fnv1a64([struct.pack("<i", mech.S), idata.astype("<i4").tobytes(), irs.astype("<i4").tobytes(),
                    dd.astype("<f8").tobytes(), np.ascontiguousarray(nasa, "<f8").tobytes(),
                    np.ascontiguousarray(W, "<f8").tobytes()])


def _f(x: float) -> str:
    return repr(float(x))


def _pow(var: str, nu: float) -> str:
    n = int(round(nu))
    if abs(nu - n) < 1e-12 and 1 <= n <= 3:
        return "*".join([var] * n)
    return f"pow({var}, {_f(nu)})"


def _dpow(var: str, nu: float) -> str:
    n = int(round(nu))
    if abs(nu - n) < 1e-12 and 1 <= n <= 3:
        return {1: "1.0", 2: f"2.0*{var}", 3: f"3.0*{var}*{var}"}[n]
    return f"{_f(nu)}*pow({var}, {_f(nu - 1)})"


def _g_rt(row, T):
    """g_i / RT of one NASA7 row at the temperatures T (array), as the generated header evaluates it."""
    a = np.where((T > row[0])[:, None], row[1:8][None, :], row[8:15][None, :])
    h = a[:, 0] + a[:, 1] / 2 * T + a[:, 2] / 3 * T ** 2 + a[:, 3] / 4 * T ** 3 + a[:, 4] / 5 * T ** 4 + a[:, 5] / T
    s = a[:, 0] * np.log(T) + a[:, 1] * T + a[:, 2] / 2 * T ** 2 + a[:, 3] / 3 * T ** 3 + a[:, 4] / 4 * T ** 4 + a[:, 6]
    return h - s


def _net_nu(mech, r):
    d = {}
    for j in range(3):
        if mech.prod[r, j] >= 0:
            d[int(mech.prod[r, j])] = d.get(int(mech.prod[r, j]), 0.0) + mech.nu_p[r, j]
        if mech.reac[r, j] >= 0:
            d[int(mech.reac[r, j])] = d.get(int(mech.reac[r, j]), 0.0) - mech.nu_r[r, j]
    return {i: v for i, v in d.items() if v != 0.0}


def _eq_product_floor(mech, nasa, rev):
    """Lowest temperature from which every reverse rate of `rev` can be formed as products of per-species
    exp(g_i / RT) (integer net coefficients): each factor and each partial product of a reaction's numerator and
    denominator stays within exp(+-600) up to 10000 K. None when some reaction never qualifies."""
    T = np.geomspace(20.0, 10000.0, 4000)
    ok = np.ones(T.size, dtype=bool)
    for r in rev:
        num = np.zeros(T.size); den = np.zeros(T.size)
        for i, v in sorted(_net_nu(mech, r).items()):
            g = _g_rt(nasa[i], T)
            for _ in range(int(round(abs(v)))):
                if v > 0:
                    num = num + g
                    ok &= np.abs(num) < 600.0
                else:
                    den = den + g
                    ok &= np.abs(den) < 600.0
            ok &= np.abs(g) < 600.0
    if not ok[-1]:
        return None
    bad = np.nonzero(~ok)[0]
    return float(T[bad[-1] + 1]) * 1.01 if bad.size else float(T[0])


def _arrhenius(A, b, Ta):
    """A T^b exp(-Ta / T) with the exponential only where it is needed (b integer or +-1/2 and Ta = 0: powers)."""
    if Ta == 0:
        n2 = 2 * b
        if b == 0:
            return _f(A)
        if abs(n2 - round(n2)) < 1e-12 and -4 <= round(n2) <= 6:
            n2 = int(round(n2))
            f = {1: "T", 2: "T2", 3: "T3", 4: "T4"}
            parts = []
            if n2 % 2:
                parts.append("sqrt(T)" if n2 > 0 else "sqrt(rT)")
            q = abs(n2) // 2
            if q:
                parts.append(f[q] if n2 > 0 else "*".join(["rT"] * q))
            return f"{_f(A)} * " + " * ".join(parts)
    return f"{_f(A)} * exp({_f(b)}*lnT - {_f(Ta)}*rT)"


def _troe_const(a, T3, T1, has_T2):
    """log10 Fc when it does not depend on T in double precision: exp(-T / T3) is exactly 0 for T3 <= 1e-30 and
    exp(-T / T1) exactly 1 for T1 >= 1e30 at every T below 1e13 K (T / T1 under half an ulp of 1). None otherwise."""
    if has_T2:
        return None
    terms = []
    for coef, Tx in ((1 - a, T3), (a, T1)):
        if Tx <= 1e-30:
            terms.append(0.0)
        elif Tx >= 1e30:
            terms.append(coef)
        else:
            return None
    return math.log10(max(terms[0] + terms[1], 1e-300))


def generate(mech, nasa, W, name: str) -> str:
    S, R = mech.S, mech.R
    nasa = np.asarray(nasa); W = np.asarray(W)
    L = []
    emit = L.append
    fp = fingerprint(mech, nasa, W)
    emit(f"// generated by dfmi/chem_codegen.py -- mechanism '{name}': S = {S}, R = {R}. Do not edit.")
    emit("// DFMI_HD is defined by the includer: __device__ in csrc/chem.hip, empty in the CPU-A baseline; so is")
    emit("// DFMI_RCP(x), 1 / x (a Newton-refined hardware reciprocal on the device, the division on the host).")
    emit(f"struct ChemGen_{name} {{")
    emit(f"  static constexpr int S = {S};")
    emit(f"  static constexpr int R = {R};")
    emit(f"  static constexpr unsigned long long FINGERPRINT = 0x{fp:016x}ull;")
    emit(f"  static constexpr double W[{S}] = {{{', '.join(_f(w) for w in W)}}};")
    emit(f"  static constexpr double RW[{S}] = {{{', '.join(_f(1.0 / w) for w in W)}}};   // 1 / W")
    # active species: a net stoichiometric change in some reaction. The others (N2 in the H2 mechanisms: a
    # third-body collider only) keep their concentration over the step, so the integrator carries them as
    # constants: their rows of w and J are zero, their columns of A multiply a zero stage increment, and
    # their error-norm terms are zero -- dropping them changes no other value.
    net = np.zeros(S, dtype=bool)
    for r in range(R):
        d = {}
        for j in range(3):
            if mech.reac[r, j] >= 0:
                d[int(mech.reac[r, j])] = d.get(int(mech.reac[r, j]), 0.0) - mech.nu_r[r, j]
            if mech.prod[r, j] >= 0:
                d[int(mech.prod[r, j])] = d.get(int(mech.prod[r, j]), 0.0) + mech.nu_p[r, j]
        for i, v in d.items():
            if v != 0.0:
                net[i] = True
    act = [i for i in range(S) if net[i]]
    apos = {i: a for a, i in enumerate(act)}
    SA = len(act)
    emit(f"  static constexpr int SA = {SA};   // active species (the integrated state)")
    emit(f"  static constexpr int ACT[SA] = {{{', '.join(str(i) for i in act)}}};")
    # ---- constants: kf[r], kr[r] (reverse = kf / Kc, 0 if irreversible), k0[r] (fall-off)
    falloff = [r for r in range(R) if mech.itype[r] >= 2]
    troe = [r for r in range(R) if mech.itype[r] == 3]
    troe_c = {r: _troe_const(mech.troe[r][0], mech.troe[r][1], mech.troe[r][2], mech.has_T2[r]) for r in troe}
    nK = 2 * R + len(falloff) + len(troe)
    emit(f"  static constexpr int NK = {nK};")
    # rate constants: k[r] forward (Arrhenius), k[R + r] reverse (= forward / Kc, 0 if irreversible), k[2R + i]
    # the fall-off low-pressure limits, then log10 Fc of the Troe reactions (a function of T alone, so it is
    # evaluated once per cell here, not in every rate evaluation; a literal where T3 / T1 make it constant -- still
    # stored with the others: read as a literal inside the rates it took the k_chem_gen wave 410 -> 418 registers,
    # past the 416 that leave a 96-VGPR assembly kernel room on the SIMD beside it); the header (ln T, 1/T, powers, Gibbs terms) is shared. Transcendentals are most of this function's
    # cost (~1,900 VALU instructions per cell for Burke 9, a third of the cell's integration): the forward rates
    # take powers instead of exp where b is a (half-)integer and Ta = 0, and above T_eq the reverse rates are
    # products of one exp(g_i / RT) per species instead of one exp per reaction
    head = ["    const double lnT = log(T), rT = 1.0 / T;",
            "    const double T2 = T * T, T3 = T2 * T, T4 = T3 * T;"]
    needs_g = sorted({int(i) for r in range(R) if mech.reversible[r]
                      for i in list(mech.reac[r]) + list(mech.prod[r]) if i >= 0})
    for i in needs_g:
        row = nasa[i]
        def hs(a):
            h = f"({_f(a[0])} + {_f(a[1] / 2)}*T + {_f(a[2] / 3)}*T2 + {_f(a[3] / 4)}*T3 + {_f(a[4] / 5)}*T4 + {_f(a[5])}*rT)"
            s = f"({_f(a[0])}*lnT + {_f(a[1])}*T + {_f(a[2] / 2)}*T2 + {_f(a[3] / 3)}*T3 + {_f(a[4] / 4)}*T4 + {_f(a[6])})"
            return f"{h} - {s}"
        head.append(f"    const double g{i} = T > {_f(row[0])} ? {hs(row[1:8])} : {hs(row[8:15])};")
    head.append(f"    const double lc = log({_f(P_ATM / RU)} * rT);   // log(p_atm / RT)")
    rev = [r for r in range(R) if mech.reversible[r]]
    # the per-species form needs integer net coefficients; a mechanism with other orders keeps the per-reaction exp
    prod_form = [r for r in rev if all(abs(v - round(v)) < 1e-12 and abs(v) <= 3 for v in _net_nu(mech, r).values())]
    T_eq = _eq_product_floor(mech, nasa, prod_form) if prod_form else None
    if T_eq is None:
        prod_form = []
    fo = {}
    kdef = {}
    kdef_eq = {}
    for r in range(R):
        lines = []
        A, b, Ta = mech.A[r], mech.b[r], mech.Ta[r]
        lines.append(f"    k[{r}] = {_arrhenius(A, b, Ta)};")
        if mech.reversible[r]:
            dG = []
            dnu = 0.0
            for j in range(3):
                if mech.prod[r, j] >= 0:
                    dG.append(f"+ {_f(mech.nu_p[r, j])}*g{mech.prod[r, j]}"); dnu += mech.nu_p[r, j]
                if mech.reac[r, j] >= 0:
                    dG.append(f"- {_f(mech.nu_r[r, j])}*g{mech.reac[r, j]}"); dnu -= mech.nu_r[r, j]
            kexp = f"    k[{R + r}] = k[{r}] * exp(0.0 {' '.join(dG)} - {_f(dnu)}*lc);"
            if r in prod_form:
                # k_r = k_f exp(sum nu g) (p_atm / RT)^-dnu = k_f prod e_i^nu_i pc^-dnu, pc = p_atm / RT
                num, den = [], []
                for i, v in sorted(_net_nu(mech, r).items()):
                    (num if v > 0 else den).extend([f"e{i}"] * int(round(abs(v))))
                n = int(round(dnu))
                (num if n < 0 else den).extend(["pc"] * abs(n))
                expr = f"k[{r}]"
                if num:
                    expr += " * (" + " * ".join(num) + ")"
                if den:
                    expr += " * DFMI_RCP(" + " * ".join(den) + ")"
                kdef_eq[r] = (f"      k[{R + r}] = {expr};", kexp.replace("    k[", "      k[", 1))
            else:
                lines.append(kexp)
        else:
            lines.append(f"    k[{R + r}] = 0.0;")
        if mech.itype[r] >= 2:
            fo[r] = 2 * R + len(fo)
            A0, b0, Ta0 = mech.A0[r], mech.b0[r], mech.Ta0[r]
            lines.append(f"    k[{fo[r]}] = {_arrhenius(A0, b0, Ta0)};")
        kdef[r] = lines
    ftroe = {}
    for r in troe:
        ftroe[r] = 2 * R + len(falloff) + len(ftroe)
        if troe_c[r] is not None:
            kdef[r].append(f"    k[{ftroe[r]}] = {_f(troe_c[r])};   // log10 Fc: T3 / T1 make it constant")
            continue
        a, T3, T1, T2 = mech.troe[r]
        fc = f"{_f(1 - a)}*exp(-T / {_f(T3)}) + {_f(a)}*exp(-T / {_f(T1)})"
        if mech.has_T2[r]:
            fc += f" + exp(-{_f(T2)} / T)"
        kdef[r].append(f"    k[{ftroe[r]}] = log10(fmax({fc}, 1e-300));   // log10 Fc")
    # k: any indexable store of the NK constants (a register array on the host / CPU-A; chem.hip passes a view
    # of the workgroup's LDS, [constant][lane], so the constants held across the step loop take no registers)
    emit("  template <class KV> DFMI_HD static inline void consts(double T, KV&& k) {")
    emit("    DFMI_CONTRACT();")   # includer-defined: FMA contraction on the device, nothing on the host
    L.extend(head)
    for r in range(R):
        L.extend(kdef[r])
    if kdef_eq:
        eq_sp = sorted({i for r in kdef_eq for i in _net_nu(mech, r)})
        emit(f"    if (T >= {_f(T_eq)}) {{   // every factor and partial product within exp(+-600) (codegen T_eq)")
        emit(f"      const double pc = {_f(P_ATM / RU)} * rT;   // p_atm / RT")
        for i in eq_sp:
            emit(f"      const double e{i} = exp(g{i});")
        for r in sorted(kdef_eq):
            emit(kdef_eq[r][0])
        emit("    } else {")
        for r in sorted(kdef_eq):
            emit(kdef_eq[r][1])
        emit("    }")
    emit("  }")
    def third_body(r):
        terms = []
        for i in range(S):
            e = mech.eff[r, i]
            if e == 0.0:
                continue
            terms.append(f"C[{i}]" if e == 1.0 else f"{_f(e)}*C[{i}]")
        return " + ".join(terms) if terms else "0.0"

    def rate_coeffs(r, out):
        """emit kf_r, kr_r (effective, incl. fall-off) and the third-body factor M_r"""
        t = mech.itype[r]
        if t == 0:
            out.append(f"    const double kf{r} = k[{r}], kr{r} = k[{R + r}];")
            return None
        out.append(f"    const double M{r} = {third_body(r)};")
        if t == 1:
            out.append(f"    const double kf{r} = k[{r}], kr{r} = k[{R + r}];")
            return f"M{r}"
        out.append(f"    const double rki{r} = DFMI_RCP(k[{r}]);")
        out.append(f"    const double Pr{r} = k[{fo[r]}] * M{r} * rki{r};")
        if t == 3:
            out.append(f"    const double lFc{r} = k[{ftroe[r]}];")
            out.append(f"    const double cc{r} = -0.4 - 0.67*lFc{r}, nn{r} = 0.75 - 1.27*lFc{r};")
            out.append(f"    const double lPr{r} = log10(fmax(Pr{r}, 1e-300));")
            out.append(f"    const double rd{r} = DFMI_RCP(nn{r} - 0.14*(lPr{r} + cc{r}));")
            out.append(f"    const double f1{r} = (lPr{r} + cc{r}) * rd{r};")
            out.append(f"    const double rg{r} = DFMI_RCP(1.0 + f1{r}*f1{r});")
            out.append(f"    const double F{r} = exp10(lFc{r} * rg{r});")
        else:
            out.append(f"    const double F{r} = 1.0;")
        out.append(f"    const double rp{r} = DFMI_RCP(1.0 + Pr{r});")
        out.append(f"    const double fo{r} = Pr{r} * rp{r} * F{r};")
        out.append(f"    const double kf{r} = k[{r}] * fo{r}, kr{r} = k[{R + r}] * fo{r};")
        return None

    def prod_terms(r):
        f = [_pow(f"C[{mech.reac[r, j]}]", mech.nu_r[r, j]) for j in range(3) if mech.reac[r, j] >= 0]
        b = [_pow(f"C[{mech.prod[r, j]}]", mech.nu_p[r, j]) for j in range(3) if mech.prod[r, j] >= 0]
        return f, b

    # ---- production rates
    emit("  template <class KV> DFMI_HD static inline void wdot(double T, const KV& k, const double (&C)[S], double (&w)[SA]) {")
    emit("    DFMI_CONTRACT();")   # includer-defined: FMA contraction on the device, nothing on the host
    emit("    (void)T;")
    acc = {i: [] for i in range(S)}
    for r in range(R):
        body = []
        M = rate_coeffs(r, body)
        L.extend(body)
        f, b = prod_terms(r)
        fwd = " * ".join([f"kf{r}"] + f)
        rev = " * ".join([f"kr{r}"] + b)
        q = f"({fwd} - {rev})" if mech.reversible[r] else f"({fwd})"
        emit(f"    const double q{r} = {M + ' * ' if M else ''}{q};")
        for j in range(3):
            if mech.reac[r, j] >= 0:
                acc[int(mech.reac[r, j])].append(f"- {_f(mech.nu_r[r, j])}*q{r}")
            if mech.prod[r, j] >= 0:
                acc[int(mech.prod[r, j])].append(f"+ {_f(mech.nu_p[r, j])}*q{r}")
    for i in act:
        emit(f"    w[{apos[i]}] = 0.0 {' '.join(acc[i])};")
    emit("  }")

    # ---- Jacobian (mass action, third-body factor, and the fall-off rate's [M]-dependence) and its pattern.
    # Fall-off: k = k_inf fo(Pr), Pr = k0 [M] / k_inf, fo = Pr / (1 + Pr) F(Pr) (Troe or F = 1), so
    # dq/dC_j gains eff_j (dfo/d[M]) (k_inf prod_f - k_inf/Kc prod_b) with
    # dfo/d[M] = (k0 / k_inf) [F / (1 + Pr)^2 + Pr / (1 + Pr) dF/dPr] and, for Troe,
    # Pr dF/dPr = -F 2 lFc f1 n / ((1 + f1^2)^2 (n - 0.14 (lPr + c))^2). Rosenbrock methods need the exact
    # Jacobian for their order; without this term the stiff flame-front cells of the 1D flame took 2-5x
    # more steps (285 vs 53 on the stiffest cell).
    jac = {}
    fused = {}
    emit("  template <class KV> DFMI_HD static inline void jac(double T, const KV& k, const double (&C)[S], "
         "double (&J)[SA * SA]) {")
    emit("    DFMI_CONTRACT();")
    emit("    (void)T;")
    for r in range(R):
        body = []
        M = rate_coeffs(r, body)
        L.extend(body)
        mark = len(L)
        f, b = prod_terms(r)
        rows = {}
        for j in range(3):
            if mech.reac[r, j] >= 0:
                rows[int(mech.reac[r, j])] = rows.get(int(mech.reac[r, j]), 0.0) - mech.nu_r[r, j]
            if mech.prod[r, j] >= 0:
                rows[int(mech.prod[r, j])] = rows.get(int(mech.prod[r, j]), 0.0) + mech.nu_p[r, j]
        rows = {i: v for i, v in rows.items() if v != 0.0}
        dq = {}
        for a in range(3):
            sp = int(mech.reac[r, a])
            if sp >= 0:
                terms = [_dpow(f"C[{sp}]", mech.nu_r[r, a])] + [f[j] for j in range(len(f)) if j != a]
                dq.setdefault(sp, []).append("+ kf%d * %s" % (r, " * ".join(terms)))
        if mech.reversible[r]:
            for a in range(3):
                sp = int(mech.prod[r, a])
                if sp >= 0:
                    terms = [_dpow(f"C[{sp}]", mech.nu_p[r, a])] + [b[j] for j in range(len(b)) if j != a]
                    dq.setdefault(sp, []).append("- kr%d * %s" % (r, " * ".join(terms)))
        if M:
            fwd = " * ".join([f"kf{r}"] + f)
            rev = " * ".join([f"kr{r}"] + b)
            q0 = f"({fwd} - {rev})" if mech.reversible[r] else f"({fwd})"
            emit(f"    const double q0_{r} = {q0};")
        if mech.itype[r] >= 2:   # fall-off: d fo / d[M] times the rate without fo
            fwd = " * ".join([f"k[{r}]"] + f)
            rev = " * ".join([f"k[{R + r}]"] + b)
            qk = f"({fwd} - {rev})" if mech.reversible[r] else f"({fwd})"
            dF = ""
            if mech.itype[r] == 3:
                dF = (f" - F{r} * 2.0 * lFc{r} * f1{r} * nn{r} * rp{r} * (rg{r} * rg{r}) * (rd{r} * rd{r})")
            emit(f"    const double dfo{r} = k[{fo[r]}] * rki{r} * (F{r} * (rp{r} * rp{r}){dF});")
            emit(f"    const double qk{r} = {qk};")
        for j in act:   # inactive columns multiply a zero increment (see SA)
            parts = []
            if j in dq:
                s = " ".join(dq[j])
                parts.append(f"{M} * (0.0 {s})" if M else f"(0.0 {s})")
            if M and mech.eff[r, j] != 0.0:
                parts.append(f"{_f(mech.eff[r, j])} * q0_{r}")
            if mech.itype[r] >= 2 and mech.eff[r, j] != 0.0:
                parts.append(f"{_f(mech.eff[r, j])} * dfo{r} * qk{r}")
            if not parts:
                continue
            emit(f"    {{ const double d = {' + '.join(parts)};")
            for i, nu in rows.items():
                emit(f"      J[{apos[i] * SA + apos[j]}] += {_f(nu)} * d;")
                jac[(apos[i], apos[j])] = True
            emit("    }")
        # the fused pass: the same body, the rate q_r and its w updates after q0_r (or after the coefficients)
        jb = L[mark:]
        fwd = " * ".join([f"kf{r}"] + f)
        rev = " * ".join([f"kr{r}"] + b)
        q = f"({fwd} - {rev})" if mech.reversible[r] else f"({fwd})"
        wupd = []
        for j in range(3):
            if mech.reac[r, j] >= 0 and int(mech.reac[r, j]) in apos:
                wupd.append(f"    w[{apos[int(mech.reac[r, j])]}] -= {_f(mech.nu_r[r, j])}*q{r};")
            if mech.prod[r, j] >= 0 and int(mech.prod[r, j]) in apos:
                wupd.append(f"    w[{apos[int(mech.prod[r, j])]}] += {_f(mech.nu_p[r, j])}*q{r};")
        if M:
            k0 = 1   # jb[0] is q0_r
            qline = [f"    const double q{r} = {M} * q0_{r};"]
        else:
            k0 = 0
            qline = [f"    const double q{r} = {q};"]
        fused[r] = body + jb[:k0] + qline + wupd + jb[k0:]
    emit("  }")
    # ---- rates and Jacobian in one pass (the ROS3 step's first evaluation): every reaction's rate coefficients
    # (third-body sum, fall-off blend) are formed once for both; w accumulates reaction by reaction in the order
    # of wdot's sums, q_r = M_r q0_r is the product wdot forms, so w and J are bitwise those of wdot + jac
    emit("  template <class KV> DFMI_HD static inline void wdot_jac(double T, const KV& k, const double (&C)[S], "
         "double (&w)[SA], double (&J)[SA * SA]) {")
    emit("    DFMI_CONTRACT();")
    emit("    (void)T;")
    for i in act:
        emit(f"    w[{apos[i]}] = 0.0;")
    for r in range(R):
        L.extend(fused[r])
        emit("    DFMI_SCHED_FENCE();")   # includer-defined: no instruction scheduled across (device), nothing (host)
    emit("  }")
    # ---- symbolic LU of A = I - hg J (no pivoting), on the structural pattern
    N = SA
    pat = {(i, j) for (i, j) in jac} | {(i, i) for i in range(N)}
    for kk in range(N):
        for i in range(kk + 1, N):
            if (i, kk) in pat:
                for j in range(kk + 1, N):
                    if (kk, j) in pat:
                        pat.add((i, j))
    nz = sorted(pat)
    emit(f"  static constexpr int NNZ_LU = {len(nz)};")
    # the factor keeps the reciprocal pivots on the diagonal (it forms them anyway to scale its columns), so the
    # three stage solves of a ROS3 step multiply instead of dividing (IEEE f64 division is ~10 VALU instructions)
    emit("  DFMI_HD static inline bool factor(double (&A)[SA * SA]) {")
    emit("    DFMI_CONTRACT();")   # includer-defined: FMA contraction on the device, nothing on the host
    for kk in range(N):
        emit(f"    if (!(fabs(A[{kk * N + kk}]) > 1e-300)) return false;")
        emit(f"    {{ const double ip = DFMI_RCP(A[{kk * N + kk}]); A[{kk * N + kk}] = ip;")
        for i in range(kk + 1, N):
            if (i, kk) not in pat:
                continue
            emit(f"      {{ const double f = A[{i * N + kk}] * ip; A[{i * N + kk}] = f;")
            for j in range(kk + 1, N):
                if (kk, j) in pat:
                    emit(f"        A[{i * N + j}] -= f * A[{kk * N + j}];")
            emit("      }")
        emit("    }")
    emit("    return true;")
    emit("  }")
    emit("  DFMI_HD static inline void solve(const double (&A)[SA * SA], double (&x)[SA]) {")
    emit("    DFMI_CONTRACT();")   # includer-defined: FMA contraction on the device, nothing on the host
    for i in range(N):
        for j in range(i):
            if (i, j) in pat:
                emit(f"    x[{i}] -= A[{i * N + j}] * x[{j}];")
    for i in range(N - 1, -1, -1):
        for j in range(i + 1, N):
            if (i, j) in pat:
                emit(f"    x[{i}] -= A[{i * N + j}] * x[{j}];")
        emit(f"    x[{i}] = x[{i}] * A[{i * N + i}];")
    emit("  }")
    emit(f"  static constexpr bool JAC_NZ[SA * SA] = {{{', '.join('true' if (i, j) in jac else 'false' for i in range(N) for j in range(N))}}};")
    emit("};")
    return "\n".join(L) + "\n"


def main(argv):
    if len(argv) != 3:
        print(__doc__)
        return 2
    path, name, out = argv
    mech = parse_mechanism(path)
    ym = read_yaml_mechanism(path)
    open(out, "w").write(generate(mech, ym["nasa"], ym["W"], name))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
