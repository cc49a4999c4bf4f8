"""The second pressure corrector preconditioned with the first corrector's V-cycle (option amg.reuse) against a
V-cycle rebuilt per solve, for the mixed-precision (fp32, face-wise level 0) and the fp64 V-cycle: both meet the
system's own tolerance (AmgX RELATIVE_INI 1e-5, amgxpOptions) in about the same number of PCG iterations and
land on the same fields to that tolerance. The fp64 V-cycle's level 0 reads the current solve's ELL values --
the reuse path must keep writing them."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, rel_err

pytestmark = pytest.mark.gpu


def _run(reuse, precision, steps=2):
    from dfmi.lib import Context, DEFAULT_OPTIONS
    from dfmi.mesh import hex_box
    from dfmi.mech import read_thermo_table, read_yaml_mechanism
    from dfmi import case
    opts = {"amg.reuse": reuse, "amg.precision": precision}
    DEFAULT_OPTIONS.update(opts)
    try:
        ym = read_yaml_mechanism(os.path.join(GOLDEN, "ES80_H2-7-16.yaml"))
        t = read_thermo_table(os.path.join(GOLDEN, "thermo_ES80_H2-7-16.txt"), ym["species"])
        m = hex_box(32, 32, 24, lengths=(2 * np.pi * 1e-3,) * 3, gradings=(1.0, 1.3, 1.0), periodic=(True,) * 3)
        ctx = Context(0)
        case.setup_context(ctx, m, t, ym["species"].index("N2"), 1e-6, case.default_patch_types(m))
        f = case.tgv_fields(m, ym["species"], kernel_radius=1.2e-3)
        case.init_state(ctx, m, t.S, f["T"], f["p"], f["U"], f["Y"])
        ctx.call("pre_time_step")
        its, rels = [], []
        for _ in range(steps):
            ctx.time_step(2)
            it, _, rel = ctx.solver_stats("p")   # the second corrector's solve
            its.append(it)
            rels.append(rel)
        out = {k: ctx.get_field(k, (m.n_cells,)) for k in ("p", "T", "rho")}
        out["U"] = ctx.get_field("U", (3, m.n_cells))
        ctx.close()
        return its, rels, out
    finally:
        for k in opts:
            DEFAULT_OPTIONS.pop(k, None)


@pytest.mark.parametrize("precision", [32, 64])
def test_reused_vcycle_meets_tolerance(precision):
    it0, rel0, a = _run(0, precision)
    it1, rel1, b = _run(1, precision)
    assert max(rel0) <= 1e-5 and max(rel1) <= 1e-5, (rel0, rel1)
    assert all(i1 <= i0 + 2 for i0, i1 in zip(it0, it1)), (it0, it1)
    assert min(it1) > 1
    # the same pressure to the solver tolerance (the p field's variation is a tiny part of its 1e5 Pa level)
    for k, tol in (("p", 1e-6), ("T", 1e-6), ("rho", 1e-6), ("U", 1e-4)):
        assert rel_err(a[k], b[k]) < tol, (k, rel_err(a[k], b[k]))
