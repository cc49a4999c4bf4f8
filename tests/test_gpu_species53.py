"""BASELINE config 4 as a dfLowMachFoam step: 53 species (SURVEY 8d synthetic GRI table, N2 last) with the
DF-ODENet surrogate as the chemistry source inside dfmi_time_step. The assembly/thermo parity of the
53-species path is in test_gpu_parity.py (fixture params gri53, gri53-walls: bitwise LDU, 1e-12
thermo, 1e-9 per-species fields after a step); here the whole loop with the surrogate runs."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def test_gri53_dnn_time_steps():
    from dfmi.mesh import hex_box
    from dfmi.mech import read_thermo_table
    from dfmi.lib import Context
    from dfmi import case
    from dfmi.synthetic import gri53_species, gri53_smooth_fractions, gri53_dnn
    sp = gri53_species(os.path.join(GOLDEN, "gri30.yaml"))
    t = read_thermo_table(os.path.join(GOLDEN, "thermo_gri53_synthetic.txt"), sp)
    m = hex_box(12, 10, 8)
    ctx = Context(0)
    case.setup_context(ctx, m, t, sp.index("N2"), 1e-6)
    gri53_dnn(ctx)
    ctx.chem_set_options(2)
    f = case.tgv_fields(m, ["H2", "O2", "N2", "H2O"], kernel_radius=1.5e-3)
    C = m.n_cells
    prog = (f["T"] - f["T"].min()) / np.ptp(f["T"])
    case.init_state(ctx, m, t.S, f["T"], f["p"], f["U"], gri53_smooth_fractions(prog, seed=2))
    ctx.call("pre_time_step")
    for _ in range(3):
        ctx.time_step(2)
    T = ctx.get_field("T", (C,))
    Y = ctx.get_field("Y", (t.S, C))
    RR = ctx.get_field("RR", (t.S, C))
    rho_old = ctx.get_field("rho_old", (C,))
    assert np.isfinite(T).all() and np.isfinite(Y).all() and np.isfinite(RR).all()
    assert T.min() > 290.0 and T.max() < 1900.0                # a smooth state stays bounded
    for e in ("U", "Y", "E"):
        it, r0, rel = ctx.solver_stats(e)
        assert it < 20 and rel <= 1e-5, (e, it, rel)           # every system met its tolerance
    it, r0, rel = ctx.solver_stats("p")
    assert it < 1000 and rel <= 1e-5, ("p", it, rel)
    assert np.abs(Y.sum(axis=0) - 1).max() < 1e-10
    hot = ctx.get_field("T", (C,)) >= 610.0
    assert np.abs(RR[:, hot]).max() > 0                   # reacting cells carry the surrogate's source
    assert ctx.dnn_stats()[0] > 0
    ctx.close()
