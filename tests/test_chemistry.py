"""Chemistry row (A10) on the CPU: mechanism parsing and the kinetics oracle's invariants.
Parity vs Cantera is unpinned (no Cantera here, no reference chemistry fixtures)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

MECHS = ["Burke2012_s9r23.yaml", "ES80_H2-7-16.yaml"]


def _kin(name):
    from dfmi.kinetics import parse_mechanism
    from dfmi.mech import read_yaml_mechanism
    from chem_oracle import Kinetics
    path = os.path.join(GOLDEN, name)
    m = parse_mechanism(path)
    ym = read_yaml_mechanism(path)
    return m, ym, Kinetics(m, ym["nasa"], ym["W"])


def _states(ym, n, seed=0):
    rng = np.random.default_rng(seed)
    sp = ym["species"]
    S = len(sp)
    Y = rng.random((S, n)) ** 3
    Y[sp.index("N2")] += 2.0
    Y /= Y.sum(axis=0)
    T = rng.uniform(300.0, 2500.0, n)
    Wm = 1.0 / (Y / ym["W"][:, None]).sum(axis=0)
    rho = 101325.0 * Wm / (8314.46261815324 * T)
    return T, rho, Y


def test_parse_burke():
    m, ym, _ = _kin(MECHS[0])
    assert (m.S, m.R) == (9, 23)
    assert list(m.itype).count(1) == 4 and list(m.itype).count(3) == 2
    assert m.reversible.all()
    sp = m.species
    # reaction 1: H + O2 <=> O + OH, A = 1.04e14 cm3/mol/s -> 1.04e11 m3/kmol/s, Ea 15286 cal/mol
    r = 0
    assert m.A[r] == pytest.approx(1.04e11) and m.Ta[r] == pytest.approx(15286 * 4.184 / 8.31446261815324)
    assert sorted(sp[i] for i in m.reac[r] if i >= 0) == ["H", "O2"]
    # three-body efficiencies and a Troe fall-off
    r = 8
    assert m.eff[r, sp.index("H2O")] == 0.0 and m.eff[r, sp.index("N2")] == 2.0
    r = 10
    assert m.itype[r] == 3 and m.troe[r, 0] == 0.5
    assert m.A0[r] == pytest.approx(6.366e20 * 1e-6)   # third order: (1e-3)^2


def test_parse_es80_units():
    m, ym, _ = _kin(MECHS[1])
    assert (m.S, m.R) == (7, 16)
    assert not m.reversible.any()                       # '=>' pairs
    assert m.A[0] == 5.5e15                             # SI file units
    assert m.Ta[0] == pytest.approx(1.033e5 * 4.184 / 8.31446261815324)


@pytest.mark.parametrize("name", MECHS)
def test_production_rates_conserve_elements(name):
    m, ym, k = _kin(name)
    T, rho, Y = _states(ym, 20)
    comp = ym["composition"]
    for c in range(20):
        C = rho[c] * Y[:, c] / ym["W"]
        w = k.production_rates(T[c], C)
        for e in ("H", "O", "N"):
            a = np.array([comp[i].get(e, 0) for i in range(m.S)])
            assert abs(a @ w) <= 1e-12 * np.abs(w).max() * a.max() + 1e-300


def test_detailed_balance_at_equilibrium():
    """Integrating long enough reaches a state where every reversible reaction is balanced."""
    m, ym, k = _kin(MECHS[0])
    T, rho, Y = _states(ym, 1, seed=3)
    T = np.array([2200.0])
    Yn = k.integrate_cell(T[0], rho[0], Y[:, 0], 1.0, rtol=1e-12, atol=1e-25)
    C = rho[0] * Yn / ym["W"]
    kf, k0, Kc = k.rate_constants(T[0])
    q = k.rates_of_progress(T[0], C)
    w = k.production_rates(T[0], C)
    assert np.abs(w).max() < 1e-8 * np.abs(C).max()
    assert abs(Yn.sum() - 1.0) < 1e-12


def test_pack_layout():
    from dfmi.kinetics import ND0
    m, _, _ = _kin(MECHS[0])
    idata, irs, dd = m.pack()
    assert idata.shape == (23, 8) and irs.shape == (23, 6) and dd.shape == (23, ND0 + 9)
    assert (idata[:, 2] == (m.reac >= 0).sum(axis=1)).all()
