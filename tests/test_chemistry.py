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


def test_heat_of_formation_weights_pinned():
    """hc_i = Hf298_i / W_i (the Qdot weights, dfChemistryModel.C:335-338) from the mechanisms' NASA7 rows
    against tabulated standard enthalpies of formation at 298.15 K (JANAF / ATcT, kJ/mol): elements in their
    reference state are 0 and the radicals and water carry their formation enthalpies."""
    from chem_oracle import hf298_per_mass
    ref = {"H2": 0.0, "O2": 0.0, "N2": 0.0, "H2O": -241.826, "H": 217.998, "O": 249.18, "OH": 37.3,
           "H2O2": -136.1, "HO2": 12.0}
    for name in MECHS:
        _, ym, _ = _kin(name)
        hc = hf298_per_mass(ym["nasa"], ym["W"])
        for i, sp in enumerate(ym["species"]):
            if sp in ref:
                kj_mol = hc[i] * ym["W"][i] / 1e6   # J/kg * kg/kmol = J/kmol -> kJ/mol
                assert abs(kj_mol - ref[sp]) < 2.5, (name, sp, kj_mol)


def test_heat_release_sums_species_in_order():
    """Qdot = -sum_i hc_i RR_i (dfChemistryModel.C:771): a closed reactor conserves mass (sum RR = 0), and the
    H2/O2 -> H2O conversion releases heat (Qdot > 0) on a hot cell."""
    from chem_oracle import heat_release, hf298_per_mass
    m, ym, kin = _kin(MECHS[0])
    T, rho, Y = _states(ym, 4, seed=3)
    T[:] = 1500.0
    RR = kin.reaction_rates(T, None, rho, Y, 1e-6)
    q = kin.heat_release(RR)
    hc = hf298_per_mass(ym["nasa"], ym["W"])
    manual = np.array([-sum(hc[i] * RR[i, c] for i in range(m.S)) for c in range(4)])
    assert np.allclose(q, manual, rtol=1e-13, atol=0)
    assert np.abs(RR.sum(axis=0)).max() < 1e-6 * np.abs(RR).max()
    assert (q > 0).all()
    assert np.array_equal(heat_release(hc, np.zeros((m.S, 3))), np.zeros(3))
