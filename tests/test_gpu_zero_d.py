"""BASELINE config 1: the reference's df0DFoam case examples/df0DFoam/zeroD_cubicReactor/H2/
cvodeIntegrator -- a 10x10x10 cube of identical 0D reactors, ES80_H2-7-16, T0 = 1000 K, p = 1 atm,
dt = 1e-6, 1000 steps (endTime 1e-3), constantProperty pressure -- on the GPU integrator through
dfmi_zero_d_step, against the oracle trajectory committed in tests/golden/zeroD_cubicReactor.json
(oracle.zero_d_trajectory, SciPy BDF at rtol 1e-14 -- converged: at 1e-12 BDF still moved the ignition
by 5 K; made by tests/golden/make_zero_d_fixture.py).

Tolerance: the GPU runs ROS3 at rtol 1e-12 / atol 1e-22 (the case asks CVODE for relTol 1e-15, which a
3rd-order one-step method does not reach in a sensible number of steps); T along the whole trajectory,
through ignition (where dT/dt peaks near 1e7 K/s), within 2e-5 relative; species within 2e-3 of their
own trajectory maximum.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def test_zero_d_trajectory_matches_oracle():
    from dfmi.mesh import hex_box
    from dfmi.mech import read_thermo_table, read_yaml_mechanism
    from dfmi.kinetics import parse_mechanism
    from dfmi.lib import Context
    from dfmi import case
    ref = json.load(open(os.path.join(GOLDEN, "zeroD_cubicReactor.json")))
    ym = read_yaml_mechanism(os.path.join(GOLDEN, ref["mechanism"]))
    sp = ym["species"]
    t = read_thermo_table(os.path.join(GOLDEN, "thermo_ES80_H2-7-16.txt"), sp)
    m = hex_box(10, 10, 10, lengths=(5e-3,) * 3, periodic=(False,) * 3)      # the case's blockMeshDict
    ctx = Context(0)
    case.setup_context(ctx, m, t, sp.index("N2"), ref["dt"])
    ctx.chem_set_mechanism(parse_mechanism(os.path.join(GOLDEN, ref["mechanism"])))
    ctx.chem_set_options(1, rtol=1e-12, atol=1e-22)
    C = m.n_cells
    Y0 = np.repeat(np.asarray(ref["Y0"])[:, None], C, axis=1)
    case.init_state(ctx, m, t.S, np.full(C, ref["T0"]), np.full(C, ref["p"]), np.zeros((3, C)), Y0)
    Tref = np.asarray(ref["T"])
    Yref = np.asarray(ref["Y"])
    n = ref["n_steps"]
    T = np.zeros(n + 1); Y = np.zeros((n + 1, t.S))
    T[0] = ref["T0"]; Y[0] = ref["Y0"]
    for k in range(1, n + 1):
        ctx.zero_d_step(ref["dt"], 1)
        Tc = ctx.get_field("T", (C,))
        assert np.ptp(Tc) <= 1e-12 * Tc[0]        # identical reactors stay identical
        T[k] = Tc[0]
        Y[k] = ctx.get_field("Y", (t.S, C))[:, 0]
    assert Tref[-1] > 2000.0                      # the oracle trajectory ignites inside the 1 ms
    assert np.abs(T - Tref).max() / Tref.max() < 2e-5, np.abs(T - Tref).max()
    scale = np.maximum(np.abs(Yref).max(axis=0), 1e-12)
    assert (np.abs(Y - Yref).max(axis=0) / scale).max() < 2e-3
    ctx.close()
