"""The V-cycle's last two levels in one workgroup (amg.hip: k_vtail, option amg.tail) must give bitwise the same
pressure solve as the launch chain it replaces (k_smooth_res_r8 + k_coarsest + k_prolong_smooth on those
levels): the same expressions in the same order, the restriction summed over the same 8 lanes."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _run(tail, dims, opts=None):
    from dfmi.lib import Context, DEFAULT_OPTIONS
    from dfmi.mesh import hex_box
    from dfmi.mech import read_thermo_table, read_yaml_mechanism
    from dfmi import case
    DEFAULT_OPTIONS["amg.tail"] = tail
    DEFAULT_OPTIONS.update(opts or {})
    try:
        ym = read_yaml_mechanism(os.path.join(GOLDEN, "ES80_H2-7-16.yaml"))
        t = read_thermo_table(os.path.join(GOLDEN, "thermo_ES80_H2-7-16.txt"), ym["species"])
        m = hex_box(*dims, lengths=(2 * np.pi * 1e-3,) * 3, gradings=(1.0, 1.3, 1.0), periodic=(True,) * 3)
        ctx = Context(0)
        case.setup_context(ctx, m, t, ym["species"].index("N2"), 1e-6, case.default_patch_types(m))
        ctx.set_solver("p", 3000, 1e-12, 1e-300)
        f = case.tgv_fields(m, ym["species"], kernel_radius=1.2e-3)
        case.init_state(ctx, m, t.S, f["T"], f["p"], f["U"], f["Y"])
        ctx.call("pre_time_step")
        ctx.kernel_timer("k_vtail")
        ctx.time_step(2)
        launches = ctx.kernel_time("k_vtail")[1]
        out = {k: ctx.get_field(k, (m.n_cells,)) for k in ("p", "T", "rho")}
        out["U"] = ctx.get_field("U", (3, m.n_cells))
        out["p_iters"] = ctx.solver_stats("p")[0]
        out["launches"] = launches
        out["levels"] = ctx.amg_info()
        ctx.close()
        return out
    finally:
        DEFAULT_OPTIONS.pop("amg.tail", None)
        for k in (opts or {}):
            DEFAULT_OPTIONS.pop(k, None)


# > 4096 cells (the batched solver, not the one-workgroup small solve); the second mesh puts a full 4096-cell
# level (four cells per thread) above the coarsest
@pytest.mark.parametrize("dims", [(20, 20, 14), (32, 32, 32)], ids=["704-cell-tail", "4096-cell-tail"])
def test_vcycle_tail_is_bitwise_the_launch_chain(dims):
    a, b = _run(1, dims), _run(0, dims)
    assert a["p_iters"] == b["p_iters"] and a["p_iters"] > 3, (a["p_iters"], b["p_iters"])
    assert a["launches"] > 0 and b["launches"] == 0, (a["launches"], b["launches"])
    for k in ("p", "T", "rho", "U"):
        assert np.array_equal(a[k], b[k]), k

