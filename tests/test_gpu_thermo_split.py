"""correctThermo split in two inside dfmi_time_step (option thermo.split): the state kernel (T, he, psi, rho) on the
main stream and the transport kernel (mu, alpha, rhoD, hai) on the side stream beside the pressure corrector,
against the fused kernel. The kernels evaluate the same expressions, but thermo_point contracts products into FMAs
at the compiler's choice, which differs between the instantiations: the mixture weight (psi) moves by an ulp, and
rhoD takes rho / p as psi in the split form (thermo.hip TH_TRANSPORT). Both runs are bitwise repeatable."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, rel_err

pytestmark = pytest.mark.gpu


def _run(split, steps):
    from dfmi.lib import Context, DEFAULT_OPTIONS
    from dfmi.mesh import hex_box
    from dfmi.mech import read_thermo_table, read_yaml_mechanism
    from dfmi import case
    DEFAULT_OPTIONS["thermo.split"] = split
    try:
        ym = read_yaml_mechanism(os.path.join(GOLDEN, "ES80_H2-7-16.yaml"))
        t = read_thermo_table(os.path.join(GOLDEN, "thermo_ES80_H2-7-16.txt"), ym["species"])
        m = hex_box(32, 32, 24, lengths=(2 * np.pi * 1e-3,) * 3, periodic=(True,) * 3)
        ctx = Context(0)
        case.setup_context(ctx, m, t, ym["species"].index("N2"), 1e-6, case.default_patch_types(m))
        f = case.tgv_fields(m, ym["species"], kernel_radius=1.2e-3)
        case.init_state(ctx, m, t.S, f["T"], f["p"], f["U"], f["Y"])
        ctx.call("pre_time_step")
        for _ in range(steps):
            ctx.time_step(2)
        C, S = m.n_cells, t.S
        out = {k: ctx.get_field(k, (C,)) for k in ("T", "he", "p", "rho", "psi", "mu", "alpha")}
        out["U"] = ctx.get_field("U", (3, C))
        for k in ("Y", "rhoD", "hai"):
            out[k] = ctx.get_field(k, (S, C))
        ctx.close()
        return out
    finally:
        DEFAULT_OPTIONS.pop("thermo.split", None)


def test_split_thermo_matches_fused_after_one_step():
    a, b = _run(0, 1), _run(1, 1)
    for k in ("T", "he", "mu", "alpha", "hai", "Y"):   # Newton T(h), transport at that T, the species solve
        assert np.array_equal(a[k], b[k]), k
    for k, tol in (("psi", 1e-15), ("rho", 1e-14), ("p", 1e-14), ("rhoD", 1e-15), ("U", 1e-10)):
        assert rel_err(a[k], b[k]) <= tol, (k, rel_err(a[k], b[k]))


def test_split_thermo_matches_fused_over_steps():
    a, b = _run(0, 3), _run(1, 3)
    for k in a:
        assert rel_err(a[k], b[k]) <= 1e-9, (k, rel_err(a[k], b[k]))
