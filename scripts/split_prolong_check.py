"""Experiment check (r06w): amg.split_prolong 1 vs 0 give bitwise the same step. Needs the experiment build (the option is not in the tree)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
from conftest import GOLDEN


def _run(split):
    from dfmi.lib import Context, DEFAULT_OPTIONS
    from dfmi.mesh import hex_box
    from dfmi.mech import read_thermo_table, read_yaml_mechanism
    from dfmi import case
    DEFAULT_OPTIONS["amg.split_prolong"] = split
    try:
        ym = read_yaml_mechanism(os.path.join(GOLDEN, "ES80_H2-7-16.yaml"))
        t = read_thermo_table(os.path.join(GOLDEN, "thermo_ES80_H2-7-16.txt"), ym["species"])
        m = hex_box(40, 40, 28, lengths=(2 * np.pi * 1e-3,) * 3, gradings=(1.0, 1.3, 1.0), periodic=(True,) * 3)
        ctx = Context(0)
        case.setup_context(ctx, m, t, ym["species"].index("N2"), 1e-6, case.default_patch_types(m))
        f = case.tgv_fields(m, ym["species"], kernel_radius=1.2e-3)
        case.init_state(ctx, m, t.S, f["T"], f["p"], f["U"], f["Y"])
        ctx.call("pre_time_step")
        ctx.time_step(3)
        out = {k: ctx.get_field(k, (m.n_cells,)) for k in ("p", "T", "rho")}
        out["p_iters"] = ctx.solver_stats("p")[0]
        ctx.close()
        return out
    finally:
        DEFAULT_OPTIONS.pop("amg.split_prolong", None)


def test_split_prolong_bitwise():
    a, b = _run(1), _run(0)
    assert a["p_iters"] == b["p_iters"] and a["p_iters"] > 3
    for k in ("p", "T", "rho"):
        assert np.array_equal(a[k], b[k]), k
