"""The reference cases' convection schemes on the GPU, bitwise against the oracle (MI355X).

div(phi,Yi_h) limitedLinear01 1 (multivariate over every Y_i and he), div(phi,K) limitedLinear 1 and
div(hDiffCorrFlux) cubic -- the schemes of the reference's own dfLowMachFoam cases
(test/dfLowMachFoam/twoD_reactingTGV/H2/cvodeSolver/system/fvSchemes:32-40), which its GPU path replaces
by upwind / linear (dfYEqn.cu:543,587-593, dfEEqn.cu:166-174). The "ll" variant selects limitedLinear 1
for Yi_h (no [0, 1] bounds, so every face's limiter comes from the on-the-fly upwind-cell gradients of all
S + 1 fields), limitedLinear01 1 for K and limitedLinearV 1 for U (the 1D flame's div(phi,U),
test/Tu500K-Phi1/system/fvSchemes). YEqn / EEqn matrices at 0 ulp, the production ELL rows at 0 ulp
against the LDU fold, one outer iteration vs the oracle's exact solves at the parity suite's tolerances.
"""
import os

import numpy as np
import pytest

from conftest import rel_err, ulp_diff
from test_gpu_parity import _case, _cmp_matrix, _ell_width

pytestmark = pytest.mark.gpu

REF = {"div(phi,Yi_h)": "Gauss limitedLinear01 1", "div(phi,K)": "Gauss limitedLinear 1",
       "div(hDiffCorrFlux)": "Gauss cubic"}
LL = {"div(phi,Yi_h)": "Gauss limitedLinear 1", "div(phi,K)": "Gauss limitedLinear01 1",
      "div(hDiffCorrFlux)": "Gauss cubic", "div(phi,U)": "Gauss limitedLinearV 1"}


def _walls(mixed=False):
    from dfmi.mesh import FIXED_VALUE, FIXED_ENERGY, GRADIENT_ENERGY, INLET_OUTLET, WAVE_TRANSMISSIVE

    def walls(m):
        fv = {}
        names = ("left",) if mixed else ("left", "right")
        fixed = [i for i, p in enumerate(m.patches) if p.name in names]
        for f in ("U", "T", "Y"):
            t = m.patch_types(0).copy()
            t[fixed] = FIXED_VALUE
            fv[f] = t
        t = m.patch_types(GRADIENT_ENERGY).copy()
        t[fixed] = FIXED_ENERGY
        fv["he"] = t
        if mixed:
            out = [i for i, p in enumerate(m.patches) if p.name == "right"]
            fv["U"][out] = INLET_OUTLET
            fv["Y"][out] = INLET_OUTLET
            fv["p"] = m.patch_types(0).copy()
            fv["p"][out] = WAVE_TRANSMISSIVE
        return fv
    return walls


@pytest.fixture(scope="module", params=["ref-periodic", "ll-periodic", "ll-walls", "ref-distorted", "ll-mixed",
                                        "ll-periodic-generic", "ll-walls-csr", "ref-gri53"])
def sc(request):
    from dfmi import lib
    p = request.param
    if p.endswith("-generic"):
        lib.DEFAULT_OPTIONS["fv.species_generic"] = 1
        request.addfinalizer(lambda: lib.DEFAULT_OPTIONS.pop("fv.species_generic", None))
    if p.endswith("-csr"):
        lib.DEFAULT_OPTIONS["fv.csr_walk"] = 1
        request.addfinalizer(lambda: lib.DEFAULT_OPTIONS.pop("fv.csr_walk", None))
    schemes = REF if p.startswith("ref") else LL
    kind = p.split("-")[1]
    if kind == "periodic":
        out = _case(mech="burke9", schemes=schemes)
    elif kind == "gri53":
        out = _case(mech="gri53", schemes=schemes)
    else:
        out = _case(periodic=False, walls=_walls(kind == "mixed"), mech="burke9", distorted=kind == "distorted",
                    mixed=kind == "mixed", schemes=schemes)
    return out + (schemes,)


def _oracle(m, t, st, pt, inert, dt, schemes):
    import oracle as O
    return O.Oracle(m, t, {k: v.copy() for k, v in st.items()}, pt, inert, 1.0 / dt, schemes=schemes)


def test_u_eqn_assembly_bitwise(sc):
    ctx, m, t, st, pt, inert, dt, schemes = sc
    from dfmi import case
    case.push_state(ctx, st)
    o = _oracle(m, t, st, pt, inert, dt, schemes)
    ref = o.u_assemble()
    ctx.assemble("U")
    res = _cmp_matrix(ctx, "U", ref, ["lower", "upper", "diag", "source", "source_solve", "internal_coeffs",
                                      "boundary_coeffs"], m.n_boundary_slots)
    bad = {k: v for k, v in res.items() if v[0] != 0}
    assert not bad, bad
    assert ulp_diff(ctx.get_field("rAU", (m.n_cells,)), o["rAU"]) == 0


def test_y_eqn_assembly_bitwise(sc):
    ctx, m, t, st, pt, inert, dt, schemes = sc
    from dfmi import case
    case.push_state(ctx, st)
    o = _oracle(m, t, st, pt, inert, dt, schemes)
    o.y_prep()
    ref = o.y_assemble()
    ctx.assemble("Y")
    res = _cmp_matrix(ctx, "Y", ref, ["lower", "upper", "diag", "source", "internal_coeffs", "boundary_coeffs"],
                      m.n_boundary_slots)
    bad = {k: v for k, v in res.items() if v[0] != 0}
    assert not bad, bad
    # the limited weights differ from upwind somewhere (the "ll" schemes), the reference's limitedLinear01
    # over a table holding he is upwind wherever he leaves [0, 1]
    up = (st["phi"] >= 0).astype(float)
    frac = float(np.mean(o["conv_w"][:m.n_faces] != up))
    if schemes is LL:
        assert frac > 0.05, frac


def test_y_ell_rows_bitwise(sc):
    ctx, m, t, st, pt, inert, dt, schemes = sc
    from dfmi import case
    case.push_state(ctx, st)
    W = _ell_width(m)
    n = t.S - 1
    ctx.assemble("Y_ell")
    got = {p: ctx.get_solver_rows("Y", p, n * (W if p == "val" else 1) * m.n_cells) for p in ("val", "dS", "rhs")}
    ctx.assemble("Y_ell_ref")
    for p in ("val", "dS", "rhs"):
        assert ulp_diff(got[p], ctx.get_solver_rows("Y", p, got[p].size)) == 0, p


def test_e_eqn_assembly_bitwise(sc):
    ctx, m, t, st, pt, inert, dt, schemes = sc
    from dfmi import case
    case.push_state(ctx, st)
    o = _oracle(m, t, st, pt, inert, dt, schemes)
    o.y_prep()
    o.energy_gradient()
    o.correct_bc("he", "he", 1)
    ref = o.e_assemble(fresh_weights=True)
    ctx.assemble("Y")
    ctx.assemble("E")
    res = _cmp_matrix(ctx, "E", ref, ["lower", "upper", "diag", "source", "internal_coeffs", "boundary_coeffs"],
                      m.n_boundary_slots)
    bad = {k: v for k, v in res.items() if v[0] != 0}
    assert not bad, bad


def test_schemes_change_the_matrices(sc):
    """the selected schemes are live: the E source differs from the reference GPU path's upwind/linear one"""
    ctx, m, t, st, pt, inert, dt, schemes = sc
    from dfmi import case
    case.push_state(ctx, st)
    o1 = _oracle(m, t, st, pt, inert, dt, schemes)
    o1.y_prep(); o1.energy_gradient(); o1.correct_bc("he", "he", 1)
    r1 = o1.e_assemble(fresh_weights=True)["source"].copy()
    o0 = _oracle(m, t, st, pt, inert, dt, None)
    o0.y_prep(); o0.energy_gradient(); o0.correct_bc("he", "he", 1)
    r0 = o0.e_assemble(fresh_weights=True)["source"].copy()
    assert rel_err(r1, r0) > 1e-12


def test_full_outer_iteration(sc):
    ctx, m, t, st, pt, inert, dt, schemes = sc
    from dfmi import case
    case.push_state(ctx, st)
    for e in ("U", "Y", "E"):
        ctx.set_solver(e, 200, 1e-15, 1e-300)
    ctx.set_solver("p", 2000, 1e-15, 1e-300)
    o = _oracle(m, t, st, pt, inert, dt, schemes)
    o.time_step(2)
    ctx.time_step(2)
    for n, tl in {"T": 1e-10, "p": 1e-11, "rho": 1e-10, "he": 1e-10}.items():
        got = ctx.get_field(n, (m.n_cells,))
        assert rel_err(got, o[n]) < tl, (n, rel_err(got, o[n]))
    assert rel_err(ctx.get_field("U", (3, m.n_cells)), o["U"]) < 1e-9
    assert rel_err(ctx.get_field("Y", (t.S, m.n_cells)), o["Y"]) < 1e-9
    assert rel_err(ctx.get_field("phi", (m.n_faces,)), o["phi"]) < 1e-9
    for e in ("U", "Y", "E"):
        ctx.set_solver(e, 20, 1e-5)
    ctx.set_solver("p", 1000, 1e-5)
    case.push_state(ctx, st)


def test_limited_v_rejected_on_processor_patches():
    """div(phi,U) limitedLinearV on a decomposed mesh is an explicit error (not silently linear); the
    other terms run decomposed (test_gpu_multirank.py::test_decomposed_case_schemes_match_single_domain)"""
    from dfmi.lib import Context, DfmiError
    from dfmi.mesh import hex_box
    from dfmi import case
    from test_gpu_parity import _mech
    ym, t = _mech("burke9")
    m = hex_box(8, 4, 4, decomp=(2, 1, 1), rank=0)
    ctx = Context(0)
    with pytest.raises(DfmiError, match="decomposed"):
        case.setup_context(ctx, m, t, ym["species"].index("N2"), 1e-6, schemes={"div(phi,U)": "limitedLinearV 1"})


def test_scheme_contract_errors():
    """dfmi_set_scheme needs the boundary initialisation (it checks the patch kinds: limitedLinearV on a
    processor patch is refused), and a limited scheme with no mesh_distance is an error, not a silent
    upwind (the limiter's d would be 0)."""
    import ctypes as C
    from dfmi.lib import Context, DfmiError, _dp
    from dfmi.mesh import hex_box
    from dfmi import case
    from test_gpu_parity import _mech
    ym, t = _mech("burke9")
    m = hex_box(6, 5, 4, lengths=(2 * np.pi * 1e-3,) * 3)
    pt = case.default_patch_types(m)
    ctx = Context(0)
    rows, cols = m.proc_rows_cols()
    ctx.set_constant_values(m.n_cells, m.n_cells, m.n_faces, m.n_boundary_slots, m.n_patches, int(rows.size),
                            m.patch_sizes, t.S, 1e6)
    ctx.set_cyclic_info(m.cyclic_neighbour())
    ctx.set_constant_indexes(m.owner, m.neighbour, rows, cols, m.global_offset)
    arrs = [np.ascontiguousarray(a, dtype=np.float64) for a in (m.sf, m.mag_sf, m.weight, m.delta_coeffs, m.volume)]
    # mesh_distance = NULL (the ABI accepts it)
    ctx._call("dfmi_init_constant_fields_internal", ctx.h, *[_dp(a) for a in arrs], None)
    with pytest.raises(DfmiError, match="dfmi_init_constant_fields_boundary"):
        ctx.set_scheme("div(phi,U)", "Gauss limitedLinearV 1")
    bsf, bmag, bdc, bw, bfc = m.boundary_arrays()
    ctx.init_constant_fields_boundary(bsf, bmag, bdc, bw, bfc, pt["calculated"], pt["extrapolated"])
    ctx.init_boundary_delta(m.boundary_delta())
    ctx.set_scheme("div(phi,Yi_h)", "Gauss limitedLinear01 1")
    for f in ("U", "p", "he", "K", "Y", "T", "rho"):
        ctx.set_patch_types(f, pt[f])
    ctx.set_inert_index(ym["species"].index("N2"))
    ctx.thermo_set_coeffs(t)
    fl = case.tgv_fields(m, ym["species"], kernel_radius=1.2e-3)
    case.init_state(ctx, m, t.S, fl["T"], fl["p"], fl["U"], fl["Y"])
    with pytest.raises(DfmiError, match="mesh_distance"):
        ctx.time_step(2)
    ctx.close()
