"""The PCG update fused with the AMG's level-0 first sweep (linsolve.hip: k_cg_x_smooth, option pcg.fuse_l0)
must give bitwise the same pressure solve as the separate k_cg_x + k_smooth_res launches: the same
residual expression for every neighbour, the same V-cycle precision and the same r.r block partials."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _run(fuse):
    from dfmi.lib import Context, DEFAULT_OPTIONS
    from dfmi.mesh import hex_box
    from dfmi.mech import read_thermo_table, read_yaml_mechanism
    from dfmi import case
    DEFAULT_OPTIONS["pcg.fuse_l0"] = fuse
    try:
        ym = read_yaml_mechanism(os.path.join(GOLDEN, "ES80_H2-7-16.yaml"))
        t = read_thermo_table(os.path.join(GOLDEN, "thermo_ES80_H2-7-16.txt"), ym["species"])
        # > 4096 cells, so the batched solver (not the one-workgroup small solve) runs
        m = hex_box(20, 20, 14, lengths=(2 * np.pi * 1e-3,) * 3, gradings=(1.0, 1.3, 1.0), periodic=(True,) * 3)
        ctx = Context(0)
        case.setup_context(ctx, m, t, ym["species"].index("N2"), 1e-6, case.default_patch_types(m))
        ctx.set_solver("p", 3000, 1e-12, 1e-300)
        f = case.tgv_fields(m, ym["species"], kernel_radius=1.2e-3)
        case.init_state(ctx, m, t.S, f["T"], f["p"], f["U"], f["Y"])
        ctx.call("pre_time_step")
        ctx.kernel_timer("k_cg_x_smooth")     # the fused launch has its own timer name
        ctx.time_step(2)
        fused_launches = ctx.kernel_time("k_cg_x_smooth")[1]
        out = {k: ctx.get_field(k, (m.n_cells,)) for k in ("p", "T", "rho")}
        out["U"] = ctx.get_field("U", (3, m.n_cells))
        out["p_iters"] = ctx.solver_stats("p")[0]
        out["fused_launches"] = fused_launches
        ctx.close()
        return out
    finally:
        DEFAULT_OPTIONS.pop("pcg.fuse_l0", None)


def test_fused_pcg_update_is_bitwise_the_separate_launches():
    a, b = _run(1), _run(0)
    assert a["p_iters"] == b["p_iters"] and a["p_iters"] > 3, (a["p_iters"], b["p_iters"])
    # the comparison means something only if the fused kernel ran in one run and not in the other
    assert a["fused_launches"] > 0 and b["fused_launches"] == 0, (a["fused_launches"], b["fused_launches"])
    for k in ("p", "T", "rho", "U"):
        assert np.array_equal(a[k], b[k]), k
