"""GPU stiff-chemistry integrator (A10) vs the CPU oracle (SciPy BDF, tight tolerances).

Semantics (dfChemistryModel::solveSingle, dfChemistryModel.C:737-780): the reactor starts from
setState_TPY(T, p, Y) -- its density is p W/(R T), not the solver's rho -- and RR is scaled by the
thermo density (problem.rhoi). The tests set rho != p W/(R T) so both roles are pinned.

RR = (Y(dt) - Y) rho / dt is a difference of nearly equal numbers, so integrator tolerances show up
amplified: with tight GPU tolerances (rtol 1e-8) RR agrees to 1e-5 of its per-species scale; with
the reference's CVODE tolerances (rtol 1e-6, atol 1e-10) to 2e-3."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _setup(mech_file, table_file, n=(8, 8, 4)):
    from dfmi.mesh import hex_box
    from dfmi.mech import read_thermo_table, read_yaml_mechanism
    from dfmi.kinetics import parse_mechanism
    from dfmi.lib import Context
    from dfmi import case
    ym = read_yaml_mechanism(os.path.join(GOLDEN, mech_file))
    t = read_thermo_table(os.path.join(GOLDEN, table_file), ym["species"])
    mech = parse_mechanism(os.path.join(GOLDEN, mech_file))
    m = hex_box(*n)
    ctx = Context(0)
    case.setup_context(ctx, m, t, ym["species"].index("N2"), 1e-6)
    ctx.chem_set_mechanism(mech)
    return ctx, m, ym, mech


def _states(ym, n, seed=0):
    rng = np.random.default_rng(seed)
    sp = ym["species"]
    from dfmi.case import h2_air_compositions
    yu, yb = h2_air_compositions(sp)
    prog = rng.random(n)
    Y = (1 - prog) * yu[:, None] + prog * yb[:, None]
    rad = rng.random((len(sp), n)) * 1e-3        # radical pool
    Y = Y + rad
    Y /= Y.sum(axis=0)
    T = 300.0 + 2200.0 * rng.random(n)
    Wm = 1.0 / (Y / ym["W"][:, None]).sum(axis=0)
    p = 101325.0 * (1.0 + 0.05 * rng.standard_normal(n))
    rho = p * Wm / (8314.46261815324 * T) * (1.0 + 0.02 * rng.standard_normal(n))   # thermo rho != reactor rho
    return T, p, rho, Y


@pytest.mark.parametrize("method", ["ros3", "ros3-generic", "extrap"])
@pytest.mark.parametrize("mech", [("Burke2012_s9r23.yaml", "thermo_Burke2012_s9r23.txt"),
                                  ("ES80_H2-7-16.yaml", "thermo_ES80_H2-7-16.txt")])
def test_chem_rr_matches_oracle(mech, method, monkeypatch):
    from chem_oracle import Kinetics
    from dfmi import lib
    monkeypatch.setitem(lib.DEFAULT_OPTIONS, "chem.method", 1 if method == "extrap" else 0)
    if method.endswith("generic"):
        monkeypatch.setitem(lib.DEFAULT_OPTIONS, "chem.generated", 0)
    ctx, m, ym, mc = _setup(*mech)
    C = m.n_cells
    T, p, rho, Y = _states(ym, C)
    ctx.set_field("T", T); ctx.set_field("p", p); ctx.set_field("rho", rho); ctx.set_field("Y", Y)
    dt = 1e-6
    kin = Kinetics(mc, ym["nasa"], ym["W"])
    idx = np.arange(0, C, 7)                     # oracle on a subset (BDF is slow in Python)
    ref = kin.reaction_rates(T[idx], p[idx], rho[idx], Y[:, idx], dt)
    # per-species scale, floored for species that do not react (N2: rounding-level RR)
    scale = np.maximum(np.abs(ref).max(axis=1, keepdims=True), 1e-3 * np.abs(ref).max())
    ctx.chem_set_options(1, rtol=1e-8, atol=1e-14)
    ctx.chem_solve(dt)
    assert ctx.get_field("chem_stats", (3, C))[:2][0].min() >= 1      # no cell hit the step limit
    if method == "ros3" and mech[0].startswith("Burke"):
        assert ctx.chem_info() == 1                               # the compiled-in mechanism ran
    rr = ctx.get_field("RR", (mc.S, C))[:, idx]
    assert np.all(np.isfinite(rr))
    assert np.abs(rr - ref).max(axis=None, initial=0) / scale.max() < 1e-5
    assert (np.abs(rr - ref) / scale).max() < 1e-4
    # mass conservation: sum_i RR_i = 0
    assert np.abs(rr.sum(axis=0)).max() < 1e-9 * np.abs(rr).max()
    ctx.chem_set_options(1, rtol=1e-6, atol=1e-10)
    ctx.chem_solve(dt)
    rr = ctx.get_field("RR", (mc.S, C))[:, idx]
    assert (np.abs(rr - ref) / scale).max() < 2e-3
    st = ctx.get_field("chem_stats", (3, C))[:2]
    assert st[0].min() >= 1


def test_chem_in_time_step():
    """mode 1 runs the integrator inside dfmi_time_step (before YEqn) and the step stays finite."""
    from dfmi import case
    ctx, m, ym, mc = _setup("Burke2012_s9r23.yaml", "thermo_Burke2012_s9r23.txt")
    f = case.tgv_fields(m, ym["species"], kernel_radius=1.5e-3, T_hot=2000.0)
    case.init_state(ctx, m, len(ym["species"]), f["T"], f["p"], f["U"], f["Y"])
    ctx.chem_set_options(1)
    ctx.call("pre_time_step")
    ctx.time_step(2)
    RR = ctx.get_field("RR", (mc.S, m.n_cells))
    T = ctx.get_field("T", (m.n_cells,))
    assert np.all(np.isfinite(RR)) and np.abs(RR).max() > 0 and np.all(np.isfinite(T))


@pytest.mark.parametrize("mech", [("Burke2012_s9r23.yaml", "thermo_Burke2012_s9r23.txt"),
                                  ("ES80_H2-7-16.yaml", "thermo_ES80_H2-7-16.txt")])
@pytest.mark.parametrize("generic", [False, True])
def test_chem_cost_binning_bitwise(mech, generic, monkeypatch):
    """Cells handed to the integrator in cost-binned order (the second solve is binned by the first
    one's step counts), over the whole mesh or inside each 4096-cell tile (three tiles, the last one
    ragged), give bitwise the results of the natural order."""
    from dfmi import lib
    if generic:
        monkeypatch.setitem(lib.DEFAULT_OPTIONS, "chem.generated", 0)
    ctx, m, ym, mc = _setup(*mech, n=(24, 24, 16))
    C = m.n_cells
    T, p, rho, Y = _states(ym, C, seed=3)
    ctx.set_field("T", T); ctx.set_field("p", p); ctx.set_field("rho", rho); ctx.set_field("Y", Y)
    ctx.chem_set_options(1)
    out = {}
    for flag in ("0", "1", "2"):
        ctx.set_option("chem.binning", int(flag))
        ctx.set_field("chem_stats", np.zeros((3, C)))   # same start: no carried step sizes
        ctx.chem_solve(1e-6)
        ctx.chem_solve(1e-6)
        assert (ctx.chem_info() > 0) != generic
        out[flag] = (ctx.get_field("RR", (mc.S, C)), ctx.get_field("chem_stats", (3, C))[:2])
    st = out["1"][1]
    assert st[0].min() >= 1 and (st[0] + st[1]).max() > (st[0] + st[1]).min()   # costs really differ
    for f in ("1", "2"):
        assert np.array_equal(out["0"][0], out[f][0])
        assert np.array_equal(out["0"][1], out[f][1])


def test_chem_density_roles():
    """The reactor density comes from (T, p, Y) -- scaling the solver rho leaves the integration alone
    -- and RR scales linearly with the thermo density it is handed."""
    ctx, m, ym, mc = _setup("Burke2012_s9r23.yaml", "thermo_Burke2012_s9r23.txt")
    C = m.n_cells
    T, p, rho, Y = _states(ym, C, seed=5)
    ctx.set_field("T", T); ctx.set_field("p", p); ctx.set_field("Y", Y)
    ctx.chem_set_options(1)
    out = []
    for f in (1.0, 1.25):
        ctx.set_field("rho", rho * f)
        ctx.set_field("chem_stats", np.zeros((3, C)))
        ctx.chem_solve(1e-6)
        out.append(ctx.get_field("RR", (mc.S, C)))
    np.testing.assert_allclose(out[1], 1.25 * out[0], rtol=1e-14, atol=0)


def test_chem_step_limit_is_an_error():
    """A cell that runs out of integrator steps makes dfmi_chem_solve (and dfmi_time_step) fail
    instead of leaving a partly integrated RR behind (chem.hip: failure counter)."""
    from dfmi.lib import DfmiError
    ctx, m, ym, mc = _setup("Burke2012_s9r23.yaml", "thermo_Burke2012_s9r23.txt")
    C = m.n_cells
    T, p, rho, Y = _states(ym, C, seed=9)
    ctx.set_field("T", T); ctx.set_field("p", p); ctx.set_field("rho", rho); ctx.set_field("Y", Y)
    ctx.chem_set_options(1, rtol=1e-10, atol=1e-16)
    ctx.chem_set_max_steps(1)
    ctx.set_field("chem_stats", np.zeros((3, C)))
    with pytest.raises(DfmiError, match="step limit"):
        ctx.chem_solve(1e-6)
    assert (ctx.get_field("chem_stats", (3, C))[0] < 0).any()
    ctx.chem_set_max_steps(100000)
    ctx.chem_set_options(1, rtol=1e-6, atol=1e-10)
    ctx.set_field("chem_stats", np.zeros((3, C)))
    ctx.chem_solve(1e-6)                      # a sufficient budget clears the error
