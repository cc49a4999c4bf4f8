"""LDS-staged YEqn preparation (fv_kernels.hip k_y_prep_brick): on a hex box in blockMesh order whose
dimensions a 16 x 4 x 4 brick divides, Y_s and alpha hai_s of the brick and its face halo are staged in LDS
and the face terms read them there. The faces, their order and every product are the face walk's, so the
prepared fields and a whole outer iteration must be bitwise those of the plain kernel (option fv.yprep_brick = 0)
-- with the species staged in two chunks (default) and all at once (=2), periodic and walled."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _run(mode, periodic, mech="burke9"):
    from dfmi.lib import Context, DEFAULT_OPTIONS
    from dfmi.mesh import hex_box
    from dfmi.mech import read_thermo_table, read_yaml_mechanism
    from dfmi import case
    files = {"burke9": ("Burke2012_s9r23.yaml", "thermo_Burke2012_s9r23.txt"),
             "es80": ("ES80_H2-7-16.yaml", "thermo_ES80_H2-7-16.txt")}[mech]
    DEFAULT_OPTIONS["fv.yprep_brick"] = mode
    try:
        ym = read_yaml_mechanism(os.path.join(GOLDEN, files[0]))
        t = read_thermo_table(os.path.join(GOLDEN, files[1]), ym["species"])
        m = hex_box(32, 8, 12, lengths=(2 * np.pi * 1e-3,) * 3, gradings=(1.0, 1.2, 1.0), periodic=(periodic,) * 3)
        ctx = Context(0)
        case.setup_context(ctx, m, t, ym["species"].index("N2"), 1e-6, case.default_patch_types(m))
        f = case.tgv_fields(m, ym["species"], kernel_radius=1.2e-3)
        case.init_state(ctx, m, t.S, f["T"], f["p"], f["U"], f["Y"])
        ctx.time_step(2)
        C, S, B = m.n_cells, t.S, m.n_boundary_slots
        out = {k: ctx.get_field(k, (m.n_cells,)) for k in ("p", "T", "rho", "he", "diffAlphaD")}
        for k in ("sumYDiffError", "hDiffCorrFlux", "U"):
            out[k] = ctx.get_field(k, (3, C))
        for k in ("boundary_sumYDiffError", "boundary_hDiffCorrFlux"):
            out[k] = ctx.get_field(k, (3, B))
        out["Y"] = ctx.get_field("Y", (S, C))
        out["hex"] = ctx.hex_dims()
        ctx.close()
        return out
    finally:
        DEFAULT_OPTIONS.pop("fv.yprep_brick", None)


@pytest.mark.parametrize("periodic", [True, False], ids=["periodic", "walls"])
@pytest.mark.parametrize("mech", ["burke9", "es80"])
def test_brick_y_prep_bitwise_face_walk(periodic, mech):
    a, b, c = _run(1, periodic, mech), _run(0, periodic, mech), _run(2, periodic, mech)
    assert a["hex"] == (32, 8, 12), a["hex"]
    for k in a:
        if k == "hex":
            continue
        assert np.array_equal(a[k], b[k]), k
        assert np.array_equal(c[k], b[k]), k
