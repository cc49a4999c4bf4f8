"""Gas-phase reaction mechanism -> the flat arrays the GPU chemistry integrator reads
(dfmi_chem_set_mechanism, include/dfmi.h).

Covers what the reference mechanisms use (Cantera YAML, PyYAML SafeLoader only): elementary
Arrhenius reactions (reversible `<=>` or irreversible `=>`), three-body reactions with collision
efficiencies, and Lindemann/Troe fall-off reactions. Units are converted to SI with kmol
(concentrations in kmol/m^3, activation energies as activation temperatures Ea/R). Reverse rates of
reversible reactions come from equilibrium constants of the NASA7 polynomials (evaluated on the
device), as in Cantera's GasKinetics.

Layout (R reactions, S species; every reaction has at most 3 reactant and 3 product entries):
  idata[R][8]: type (0 elementary, 1 three-body, 2 Lindemann, 3 Troe), reversible,
               n_reactants, n_products, has_T2, 0, 0, 0
  irs[R][6]:   reactant species ids (3, -1 padded), product species ids (3)
  ddata[R][NDR]: A, b, Ta, nu_r[3], nu_p[3], A0, b0, Ta0, troe_A, T3, T1, T2, eff[S]
"""
from __future__ import annotations

import re
from dataclasses import dataclass

import numpy as np
import yaml

R_CAL = 4.184                       # J/cal
R_UNIV_MOL = 8.31446261815324      # J/mol/K
ND0 = 17                            # fixed doubles per reaction before the S efficiencies


@dataclass
class Mechanism:
    species: list
    S: int
    R: int
    itype: np.ndarray      # [R]
    reversible: np.ndarray  # [R]
    reac: np.ndarray       # [R,3] species id or -1
    prod: np.ndarray       # [R,3]
    nu_r: np.ndarray       # [R,3]
    nu_p: np.ndarray       # [R,3]
    A: np.ndarray          # SI kmol units
    b: np.ndarray
    Ta: np.ndarray         # K
    A0: np.ndarray         # low-pressure limit (fall-off)
    b0: np.ndarray
    Ta0: np.ndarray
    troe: np.ndarray       # [R,4] A, T3, T1, T2
    has_T2: np.ndarray
    eff: np.ndarray        # [R,S] third-body efficiencies (1 default)

    def pack(self):
        idata = np.zeros((self.R, 8), np.int32)
        idata[:, 0] = self.itype
        idata[:, 1] = self.reversible
        idata[:, 2] = (self.reac >= 0).sum(axis=1)
        idata[:, 3] = (self.prod >= 0).sum(axis=1)
        idata[:, 4] = self.has_T2
        irs = np.concatenate([self.reac, self.prod], axis=1).astype(np.int32)
        d = np.zeros((self.R, ND0 + self.S))
        d[:, 0] = self.A; d[:, 1] = self.b; d[:, 2] = self.Ta
        d[:, 3:6] = self.nu_r; d[:, 6:9] = self.nu_p
        d[:, 9] = self.A0; d[:, 10] = self.b0; d[:, 11] = self.Ta0
        d[:, 12:16] = self.troe
        d[:, ND0:] = self.eff
        return np.ascontiguousarray(idata), np.ascontiguousarray(irs), np.ascontiguousarray(d)


_UNIT_LEN = {"m": 1.0, "cm": 1e-2, "mm": 1e-3}
_UNIT_QTY = {"kmol": 1.0, "mol": 1e-3, "molec": 1.0 / 6.02214076e26}
_UNIT_E = {"J/kmol": 1.0, "J/mol": 1e3, "cal/mol": R_CAL * 1e3, "kcal/mol": R_CAL * 1e6, "K": None}


def _side(expr: str):
    """'2 H + O2' -> {'H': 2.0, 'O2': 1.0}; strips '+ M' / '(+ M)'."""
    expr = expr.replace("(+M)", "").replace("(+ M)", "")
    out = {}
    for tok in expr.split(" + "):
        tok = tok.strip()
        if not tok or tok == "M":
            continue
        m = re.match(r"^(\d+(?:\.\d*)?)\s+(\S+)$", tok)
        if m:
            n, sp = float(m.group(1)), m.group(2)
        else:
            n, sp = 1.0, tok
        out[sp] = out.get(sp, 0.0) + n
    return out


def _energy_to_K(v, default_unit):
    """activation energy (number or 'value unit' string) -> activation temperature [K]"""
    if isinstance(v, str):
        num, unit = v.split()
        v, unit = float(num), unit
    else:
        v, unit = float(v), default_unit
    if unit == "K":
        return v
    return v * _UNIT_E[unit] / (R_UNIV_MOL * 1e3)


def parse_mechanism(path: str) -> Mechanism:
    with open(path) as f:
        doc = yaml.load(f, Loader=yaml.SafeLoader)
    units = doc.get("units", {})
    L = _UNIT_LEN[units.get("length", "m")]
    Q = _UNIT_QTY[units.get("quantity", "kmol")]
    Eu = units.get("activation-energy", "J/kmol")
    phase = doc["phases"][0]
    species = list(phase["species"])
    S = len(species)
    sid = {s: i for i, s in enumerate(species)}
    rx = doc.get("reactions", [])
    R = len(rx)
    mk = lambda *shape, v=0.0: np.full(shape, v)
    itype = np.zeros(R, np.int32); rev = np.zeros(R, np.int32)
    reac = -np.ones((R, 3), np.int32); prod = -np.ones((R, 3), np.int32)
    nu_r = mk(R, 3); nu_p = mk(R, 3)
    A = mk(R); b = mk(R); Ta = mk(R); A0 = mk(R); b0 = mk(R); Ta0 = mk(R)
    troe = mk(R, 4); hasT2 = np.zeros(R, np.int32); eff = mk(R, S, v=1.0)
    # concentration unit conversion: (qty / length^3) -> kmol/m^3
    cfac = Q / L ** 3

    def conv_A(a, order):
        # A [conc^(1-order) / s] in file units -> SI kmol units
        return float(a) * cfac ** (1.0 - order)

    for r, x in enumerate(rx):
        eq = x["equation"]
        if "<=>" in eq:
            lhs, rhs = eq.split("<=>"); rev[r] = 1
        elif "=>" in eq:
            lhs, rhs = eq.split("=>"); rev[r] = 0
        else:
            lhs, rhs = eq.split("="); rev[r] = 1
        if x.get("reversible") is False:
            rev[r] = 0
        typ = x.get("type", "elementary")
        lr, rr = _side(lhs), _side(rhs)
        if len(lr) > 3 or len(rr) > 3:
            raise ValueError(f"reaction {r}: more than 3 distinct reactants/products")
        for k, (sp, n) in enumerate(lr.items()):
            reac[r, k] = sid[sp]; nu_r[r, k] = n
        for k, (sp, n) in enumerate(rr.items()):
            prod[r, k] = sid[sp]; nu_p[r, k] = n
        order = sum(lr.values())
        if typ in ("three-body",):
            itype[r] = 1
            rc = x["rate-constant"]
            A[r] = conv_A(rc["A"], order + 1); b[r] = float(rc["b"]); Ta[r] = _energy_to_K(rc["Ea"], Eu)
        elif typ == "falloff":
            lo, hi = x["low-P-rate-constant"], x["high-P-rate-constant"]
            A[r] = conv_A(hi["A"], order); b[r] = float(hi["b"]); Ta[r] = _energy_to_K(hi["Ea"], Eu)
            A0[r] = conv_A(lo["A"], order + 1); b0[r] = float(lo["b"]); Ta0[r] = _energy_to_K(lo["Ea"], Eu)
            if "Troe" in x:
                itype[r] = 3
                t = x["Troe"]
                troe[r] = [float(t["A"]), float(t["T3"]), float(t["T1"]), float(t.get("T2", 0.0))]
                hasT2[r] = 1 if "T2" in t else 0
            else:
                itype[r] = 2
        elif typ == "elementary":
            itype[r] = 0
            rc = x["rate-constant"]
            A[r] = conv_A(rc["A"], order); b[r] = float(rc["b"]); Ta[r] = _energy_to_K(rc["Ea"], Eu)
        else:
            raise ValueError(f"reaction {r}: type '{typ}' not supported")
        if itype[r] != 0:
            for sp, e in (x.get("efficiencies") or {}).items():
                if sp in sid:
                    eff[r, sid[sp]] = float(e)
            if "default-efficiency" in x:
                d = float(x["default-efficiency"])
                for i, sp in enumerate(species):
                    if sp not in (x.get("efficiencies") or {}):
                        eff[r, i] = d
    return Mechanism(species, S, R, itype, rev, reac, prod, nu_r, nu_p, A, b, Ta, A0, b0, Ta0, troe, hasT2, eff)
