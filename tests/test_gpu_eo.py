"""Even-odd (red-black) reduced BiCGStab for the U / Y / E systems (linsolve.hip k_eo_*).

On a coupling graph that 2-colours (hex meshes: walled, or periodic with even cyclic extents) the
Jacobi-scaled system is solved on the colour-1 Schur complement and colour 0 is recovered afterwards.
Same stopping test as the Jacobi path (AmgX RELATIVE_INI_CORE on the full residual): at tight tolerances
one outer iteration reaches the oracle's exact solves (the same 1e-9..1e-11 bounds as
test_gpu_parity.test_full_outer_iteration); at production tolerances it needs no more iterations than the
Jacobi path (option solver.even_odd = 0) and agrees with it to the solver tolerance; it is bitwise repeatable. A mesh
that does not 2-colour (a periodic direction of odd extent) keeps the Jacobi path.
The layout is decided when the gather rows are built, so the environment is set before the context
exists; solver.small = 0 keeps these small meshes off the one-workgroup path.
"""
import numpy as np
import pytest

from conftest import rel_err, ulp_diff
from test_gpu_parity import _case, _oracle, _ell_width

pytestmark = pytest.mark.gpu


def _walls(m):
    from dfmi.mesh import FIXED_VALUE, FIXED_ENERGY, GRADIENT_ENERGY
    fixed = [i for i, p in enumerate(m.patches) if p.name in ("left", "right")]
    fv = {}
    for f in ("U", "T", "Y"):
        t = m.patch_types(0).copy()
        t[fixed] = FIXED_VALUE
        fv[f] = t
    t = m.patch_types(GRADIENT_ENERGY).copy()
    t[fixed] = FIXED_ENERGY
    fv["he"] = t
    return fv


CASES = {
    # (kwargs of _case, expect the even-odd path)
    "periodic-even": (dict(nx=16, ny=12, nz=8, mech="burke9"), True),
    "walls-odd": (dict(nx=15, ny=11, nz=7, periodic=False, walls=_walls, mech="burke9"), True),   # ne != no
    "distorted": (dict(periodic=False, walls=_walls, distorted=True, mech="burke9"), True),
    "periodic-odd": (dict(nx=15, ny=12, nz=8, mech="burke9"), False),   # x cycle of odd length: no 2-colouring
}


def _make(name, monkeypatch, eo=True):
    from dfmi import lib
    monkeypatch.setitem(lib.DEFAULT_OPTIONS, "solver.small", 0)
    monkeypatch.setitem(lib.DEFAULT_OPTIONS, "solver.even_odd", 1 if eo else 0)
    kw, _ = CASES[name]
    return _case(**kw)


def _step(ctx, m, t, st, tight):
    from dfmi import case
    case.push_state(ctx, st)
    if tight:
        for e in ("U", "Y", "E"):
            ctx.set_solver(e, 300, 1e-15, 1e-300)
        ctx.set_solver("p", 3000, 1e-15, 1e-300)
    else:
        for e in ("U", "Y", "E"):
            ctx.set_solver(e, 20, 1e-5)
        ctx.set_solver("p", 1000, 1e-5)
    ctx.kernel_timer("k_bcg_eo")
    ctx.time_step(2)
    n_eo = ctx.kernel_time("k_bcg_eo")[1]
    ctx.kernel_timer("")
    out = {n: ctx.get_field(n, (m.n_cells,)) for n in ("T", "p", "rho", "he")}
    out["U"] = ctx.get_field("U", (3, m.n_cells))
    out["Y"] = ctx.get_field("Y", (t.S, m.n_cells))
    its = {e: ctx.solver_stats(e)[0] for e in ("U", "Y", "E", "p")}
    return out, its, n_eo


@pytest.mark.parametrize("name", list(CASES))
def test_eo_full_step_matches_oracle(name, monkeypatch):
    ctx, m, t, st, pt, inert, dt = _make(name, monkeypatch)
    o = _oracle(m, t, st, pt, inert, dt)
    o.time_step(2)
    out, its, n_eo = _step(ctx, m, t, st, tight=True)
    assert (n_eo > 0) == CASES[name][1], (name, n_eo)
    for n, tl in {"T": 1e-10, "p": 1e-11, "rho": 1e-10, "he": 1e-10}.items():
        assert rel_err(out[n], o[n]) < tl, (n, rel_err(out[n], o[n]))
    assert rel_err(out["U"], o["U"]) < 1e-9
    assert rel_err(out["Y"], o["Y"]) < 1e-9
    ctx.close()


@pytest.mark.parametrize("name", ["periodic-even", "walls-odd"])
def test_eo_vs_jacobi_production_tolerances(name, monkeypatch):
    """Same stopping test: the reduced solve never needs more iterations than the Jacobi path and lands
    within the tolerance's reach of it; two runs are bitwise identical."""
    ctx, m, t, st, pt, inert, dt = _make(name, monkeypatch, eo=True)
    a, its_eo, n_eo = _step(ctx, m, t, st, tight=False)
    b, _, _ = _step(ctx, m, t, st, tight=False)
    assert n_eo > 0
    for n in a:
        assert ulp_diff(a[n], b[n]) == 0, n       # run-to-run determinism (fixed-order reductions)
    ctx.close()
    ctx, m, t, st, pt, inert, dt = _make(name, monkeypatch, eo=False)
    c, its_jac, n_jac = _step(ctx, m, t, st, tight=False)
    assert n_jac == 0
    ctx.close()
    for e in ("U", "Y", "E"):
        assert its_eo[e] <= its_jac[e], (e, its_eo, its_jac)
    assert its_eo["Y"] < its_jac["Y"], (its_eo, its_jac)
    for n in ("T", "p", "rho"):
        assert rel_err(a[n], c[n]) < 1e-6, (n, rel_err(a[n], c[n]))
    assert rel_err(a["U"], c["U"]) < 1e-4
    assert rel_err(a["Y"], c["Y"]) < 1e-4


def test_eo_solver_rows_bitwise(monkeypatch):
    """The production YEqn rows written in the even-odd row order equal the LDU fold written in the same
    order; dfmi_get_solver_rows returns them in cell order."""
    ctx, m, t, st, pt, inert, dt = _make("periodic-even", monkeypatch)
    W = _ell_width(m)
    n = t.S - 1
    ctx.time_step(2)          # builds the rows' layout
    from dfmi import case
    case.push_state(ctx, st)
    ctx.assemble("Y_ell")
    got = {p: ctx.get_solver_rows("Y", p, n * (W if p == "val" else 1) * m.n_cells) for p in ("val", "dS", "rhs")}
    ctx.assemble("Y_ell_ref")
    for p in ("val", "dS", "rhs"):
        ref = ctx.get_solver_rows("Y", p, got[p].size)
        assert ulp_diff(got[p], ref) == 0, p
        assert np.abs(ref).max() > 0, p
    ctx.close()
    # in cell order they are the rows the Jacobi path's natural layout holds
    ctx, m, t, st, pt, inert, dt = _make("periodic-even", monkeypatch, eo=False)
    ctx.time_step(2)
    case.push_state(ctx, st)
    ctx.assemble("Y_ell")
    for p in ("val", "dS", "rhs"):
        assert ulp_diff(got[p], ctx.get_solver_rows("Y", p, got[p].size)) == 0, p
    ctx.close()
