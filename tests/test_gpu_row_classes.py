"""Row classes (linsolve.hip build_ell, dfmi_common.h ColView): on a hex box in blockMesh order every
gather row is one of 27 (column offset, coefficient source) patterns, so the solver SpMVs, the AMG level-0
sweeps and the assembly face loops decode a cell's row from one byte instead of reading 2 W explicit ints.
The decoded columns and sources are the explicit ones, so a whole outer iteration must be bitwise the run
with the option solver.row_classes = 0 -- periodic (cyclic partner offsets in the table), walled (padding entries) and
decomposed (processor halo columns read explicitly) meshes."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _run(classes, periodic, env=None):
    from dfmi.lib import Context, DEFAULT_OPTIONS
    from dfmi.mesh import hex_box
    from dfmi.mech import read_thermo_table, read_yaml_mechanism
    from dfmi import case
    DEFAULT_OPTIONS["solver.row_classes"] = classes
    for k, v in (env or {}).items():
        DEFAULT_OPTIONS[k] = v
    try:
        ym = read_yaml_mechanism(os.path.join(GOLDEN, "ES80_H2-7-16.yaml"))
        t = read_thermo_table(os.path.join(GOLDEN, "thermo_ES80_H2-7-16.txt"), ym["species"])
        # > 4096 cells: the batched solvers (not the one-workgroup small solves) run
        m = hex_box(20, 18, 14, lengths=(2 * np.pi * 1e-3,) * 3, gradings=(1.0, 1.3, 1.0), periodic=(periodic,) * 3)
        ctx = Context(0)
        case.setup_context(ctx, m, t, ym["species"].index("N2"), 1e-6, case.default_patch_types(m))
        f = case.tgv_fields(m, ym["species"], kernel_radius=1.2e-3)
        case.init_state(ctx, m, t.S, f["T"], f["p"], f["U"], f["Y"])
        ctx.time_step(2)
        out = {k: ctx.get_field(k, (m.n_cells,)) for k in ("p", "T", "rho", "he")}
        out["U"] = ctx.get_field("U", (3, m.n_cells))
        out["Y"] = ctx.get_field("Y", (t.S, m.n_cells))
        out["iters"] = {e: ctx.solver_stats(e)[0] for e in ("U", "Y", "E", "p")}
        out["ncls"] = ctx.row_classes()
        out["hex"] = ctx.hex_dims()
        ctx.close()
        return out
    finally:
        DEFAULT_OPTIONS.pop("solver.row_classes", None)
        for k in (env or {}):
            DEFAULT_OPTIONS.pop(k, None)


@pytest.mark.parametrize("periodic", [True, False], ids=["periodic", "walls"])
def test_row_classes_bitwise_explicit_rows(periodic):
    a, b = _run(1, periodic), _run(0, periodic)
    assert b["ncls"] == 0 and 1 < a["ncls"] <= 27, (a["ncls"], b["ncls"])
    assert a["iters"] == b["iters"], (a["iters"], b["iters"])
    for k in ("p", "T", "rho", "he", "U", "Y"):
        assert np.array_equal(a[k], b[k]), k


@pytest.mark.parametrize("periodic", [True, False], ids=["periodic", "walls"])
def test_hex_face_walk_bitwise_explicit_rows(periodic):
    """the computed hex face walk (each_face<-1>) against the ELL-row and CSR walks: bitwise"""
    a = _run(1, periodic)
    b = _run(1, periodic, {"fv.hex_walk": 0})
    c = _run(1, periodic, {"fv.hex_walk": 0, "fv.csr_walk": 1})
    assert a["hex"] == (20, 18, 14), a["hex"]
    assert a["iters"] == b["iters"] == c["iters"], (a["iters"], b["iters"], c["iters"])
    for k in ("p", "T", "rho", "he", "U", "Y"):
        assert np.array_equal(a[k], b[k]) and np.array_equal(a[k], c[k]), k


@pytest.mark.parametrize("periodic", [True, False], ids=["periodic", "walls"])
def test_face_form_pressure_operator_bitwise_ell(periodic):
    """the symmetric p operator read face-wise (FaceOp: PCG SpMVs and the fp32 AMG level 0 from the face and
    slot coefficients) against the ELL values: the same entries in the same order, so bitwise"""
    a = _run(1, periodic)
    b = _run(1, periodic, {"pcg.face_form": 0})
    assert a["iters"] == b["iters"], (a["iters"], b["iters"])
    for k in ("p", "T", "rho", "he", "U", "Y"):
        assert np.array_equal(a[k], b[k]), k
