"""BASELINE config 3 at its full size (128^3 = 2,097,152 cells, the reference TGV fields tiled, Burke 9
species, ROS3 chemistry, the convection schemes the bench runs -- the case's fvSchemes -- and the GPU reference's
upwind/linear), checked through properties that do not need the oracle at this size:

- determinism: the same state stepped twice gives bitwise identical fields (no floating-point atomics,
  fixed-order reductions) -- the property that makes the bitwise oracle tests meaningful at scale;
- discrete conservation: rhoEqn on a periodic box changes the total mass only by rounding
  (sum over cells of the face-flux divergence vanishes), species sum to 1 in every cell, T stays in
  the physical range and the solvers meet their tolerance.
"""
import os
import sys

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu


def _headline(n=128, schemes="case"):
    """the bench's workload: its mesh, state, chemistry and convection schemes (bench.py --schemes: the
    case's own fvSchemes -- limitedLinear01 / limitedLinear / cubic -- or the GPU reference's upwind/linear)"""
    sys.path.insert(0, ROOT)
    from bench import MECHS, reference_fields, case_schemes, gpu_schemes
    from dfmi.mesh import hex_box
    from dfmi.mech import read_thermo_table, read_yaml_mechanism
    from dfmi.kinetics import parse_mechanism
    from dfmi.lib import Context
    from dfmi import case
    ym = read_yaml_mechanism(os.path.join(GOLDEN, MECHS["burke9"][0]))
    t = read_thermo_table(os.path.join(GOLDEN, MECHS["burke9"][1]), ym["species"])
    m = hex_box(n, n, n, lengths=(2 * np.pi * 1e-3,) * 3)
    ctx = Context(0)
    case.setup_context(ctx, m, t, ym["species"].index("N2"), 1e-6,
                       schemes=case_schemes() if schemes == "case" else gpu_schemes())
    ctx.chem_set_mechanism(parse_mechanism(os.path.join(GOLDEN, MECHS["burke9"][0])))
    ctx.chem_set_options(1, rtol=1e-6, atol=1e-10)
    f = reference_fields(m, ym["species"])
    case.init_state(ctx, m, t.S, f["T"], f["p"], f["U"], f["Y"])
    return ctx, m, t


MAX_ITERS = {"U": 20, "Y": 20, "E": 20, "p": 1000}   # AmgX maxIters of amgx{U,Y,E,p}Options (capi.cpp:82)


def _assert_converged(ctx):
    """every system of the last solve of each equation met the relative tolerance (1e-5 of the initial
    residual, AmgX RELATIVE_INI) before the iteration cap: a solve that stopped at maxIters fails"""
    for e, cap in MAX_ITERS.items():
        it, r0, rel = ctx.solver_stats(e)
        assert it < cap and rel <= 1e-5, (e, it, r0, rel)


@pytest.mark.parametrize("schemes", ["case", "gpu"])
def test_full_size_steps_are_deterministic_and_conservative(schemes):
    from dfmi import case
    ctx, m, t = _headline(schemes=schemes)
    C, S = m.n_cells, t.S
    ctx.time_step(2)                                   # develop the state a little
    st = case.pull_state(ctx, m, S)
    runs = []
    ctx.kernel_timer("k_bcg_eo")
    for _ in range(2):
        case.push_state(ctx, st)
        ctx.set_field("chem_stats", np.zeros((3, C)))
        ctx.time_step(2)
        runs.append({n: ctx.get_field(n, (C,)) for n in ("T", "p", "rho", "he")} |
                    {"U": ctx.get_field("U", (3, C)), "Y": ctx.get_field("Y", (S, C))})
    assert ctx.kernel_time("k_bcg_eo")[1] > 0          # the even-odd BiCGStab ran (the 2-colourable box)
    ctx.kernel_timer("")
    for k in runs[0]:
        assert np.array_equal(runs[0][k], runs[1][k]), k
    T, Y = runs[0]["T"], runs[0]["Y"]
    assert np.isfinite(T).all() and 290.0 < T.min() and T.max() < 2600.0
    assert np.abs(Y.sum(axis=0) - 1.0).max() < 1e-12 and Y.min() >= 0.0
    _assert_converged(ctx)
    # rhoEqn alone: sum(rho V) is conserved on the periodic box (divergence of the face fluxes sums to 0)
    ctx.call("pre_time_step")
    rho_old = ctx.get_field("rho_old", (C,))
    ctx.call("rho_process")
    rho = ctx.get_field("rho", (C,))
    V = m.volume
    assert abs(np.sum(rho * V) - np.sum(rho_old * V)) <= 1e-13 * np.sum(rho_old * V)
    assert np.abs(rho - rho_old).max() > 0.0           # the fluxes were not zero
    ctx.close()


def test_config4_full_size_deterministic_and_closed():
    """BASELINE config 4 at its full size (128^3 cells x 53 species, synthetic GRI table, the DF-ODENet
    source of 52 nets [55,1600,800,400,1] on MFMA fp16): the large-mechanism kernels (species-chunked Y
    assembly, cooperative thermo, batched 52-system BiCGStab, compacted DNN inference) give bitwise
    identical fields when the same state is stepped twice, species close to 1 in every cell, T stays
    physical and every solve meets its tolerance. Run with the case's convection schemes, as the bench's
    config-4 line (bench.py config4_line) runs it."""
    sys.path.insert(0, ROOT)
    from bench import MECHS, reference_fields, case_schemes
    from dfmi.mesh import hex_box
    from dfmi.mech import read_thermo_table, read_yaml_mechanism
    from dfmi.lib import Context
    from dfmi import case
    from dfmi.synthetic import gri53_species, gri53_smooth_fractions, gri53_dnn
    n = 128
    m = hex_box(n, n, n, lengths=(2 * np.pi * 1e-3,) * 3)
    f = reference_fields(m, read_yaml_mechanism(os.path.join(GOLDEN, MECHS["burke9"][0]))["species"])
    sp = gri53_species(os.path.join(GOLDEN, "gri30.yaml"))
    t = read_thermo_table(os.path.join(GOLDEN, "thermo_gri53_synthetic.txt"), sp)
    ctx = Context(0)
    case.setup_context(ctx, m, t, sp.index("N2"), 1e-6, schemes=case_schemes())
    gri53_dnn(ctx)
    ctx.chem_set_options(2)
    T0 = f["T"]
    case.init_state(ctx, m, t.S, T0, f["p"], f["U"], gri53_smooth_fractions((T0 - T0.min()) / max(np.ptp(T0), 1.0)))
    C, S = m.n_cells, t.S
    ctx.time_step(2)
    assert ctx.dnn_stats()[0] > 0                      # the hot kernel reacts
    st = case.pull_state(ctx, m, S)
    runs = []
    for _ in range(2):
        case.push_state(ctx, st)
        ctx.time_step(2)
        runs.append({k: ctx.get_field(k, (C,)) for k in ("T", "p", "rho", "he")} |
                    {"U": ctx.get_field("U", (3, C)), "Y": ctx.get_field("Y", (S, C))})
    for k in runs[0]:
        assert np.array_equal(runs[0][k], runs[1][k]), k
    T, Y = runs[0]["T"], runs[0]["Y"]
    assert np.isfinite(T).all() and 250.0 < T.min() and T.max() < 3000.0
    assert np.abs(Y.sum(axis=0) - 1.0).max() < 1e-12 and Y.min() >= 0.0
    _assert_converged(ctx)
    ctx.close()
