"""Transport-fit generator (dfmi.transport_fit) pinned against the table the reference ships for
ES80_H2-7-16 (generated there with Cantera). Tolerances are the stated difference of our collision
integrals (Neufeld correlations + Brokaw dipole correction) from Cantera's Monchick-Mason tables:
non-polar species <= 0.6 %, the strongly polar H2O <= 5 %, binary diffusion <= 3 %."""
import os

import numpy as np

from conftest import GOLDEN


def _eval(c, T):
    L = np.log(T)
    return sum(c[i] * L ** i for i in range(5))


def test_es80_fits_match_reference_table(es80):
    from dfmi.transport_fit import fit_mechanism
    ref, ym = es80
    t = fit_mechanism(ym)
    assert np.array_equal(t.nasa, ref.nasa) and np.allclose(t.W, ref.W)
    T = np.linspace(300.0, 3000.0, 40)
    for k, s in enumerate(ym["species"]):
        mu_r = _eval(ref.visc[k], T) ** 2 * np.sqrt(T); mu = _eval(t.visc[k], T) ** 2 * np.sqrt(T)
        la_r = _eval(ref.cond[k], T) * np.sqrt(T); la = _eval(t.cond[k], T) * np.sqrt(T)
        tol = 0.05 if s == "H2O" else 0.006
        assert np.abs(mu / mu_r - 1).max() < tol, s
        assert np.abs(la / la_r - 1).max() < tol, s
    for k in range(t.S):
        for j in range(t.S):
            d_r = _eval(ref.bdiff[k, j], T); d = _eval(t.bdiff[k, j], T)
            assert np.abs(d / d_r - 1).max() < 0.03, (k, j)
            assert np.array_equal(t.bdiff[k, j], t.bdiff[j, k])


def test_burke9_table_is_reproducible_and_sane():
    from dfmi.mech import read_yaml_mechanism, read_thermo_table
    from dfmi.transport_fit import fit_mechanism
    ym = read_yaml_mechanism(os.path.join(GOLDEN, "Burke2012_s9r23.yaml"))
    committed = read_thermo_table(os.path.join(GOLDEN, "thermo_Burke2012_s9r23.txt"), ym["species"])
    t = fit_mechanism(ym)
    assert t.S == 9 and ym["species"] == ["H", "H2", "O", "OH", "H2O", "O2", "HO2", "H2O2", "N2"]
    for a, b in ((t.visc, committed.visc), (t.cond, committed.cond), (t.bdiff, committed.bdiff)):
        assert np.allclose(a, b, rtol=1e-12, atol=0)
    T = np.array([300.0, 1000.0, 2500.0])
    n2 = ym["species"].index("N2")
    mu = _eval(t.visc[n2], T) ** 2 * np.sqrt(T)
    assert np.all(np.diff(mu) > 0) and 1.5e-5 < mu[0] < 2.0e-5
