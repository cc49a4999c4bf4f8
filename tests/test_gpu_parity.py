"""HIP path vs CPU oracle parity (MI355X). Calls go through the C ABI (libdfmi.so).

Assembly stages are compared bit-for-bit (the HIP kernels reproduce the oracle's operation
sequence; tolerance 0 ulp, reported as max ulp); the thermo stage (log/sqrt/pow on device vs
glibc) at 1e-12 relative; a full outer iteration at 1e-9 relative with tight solver tolerances
(the reference's own tolerances are 1e-14 for LDU and 1e-10 for fields).
"""
import os

import numpy as np
import pytest

from conftest import rel_err, ulp_diff, GOLDEN

pytestmark = pytest.mark.gpu


MECHS = {"es80": ("ES80_H2-7-16.yaml", "thermo_ES80_H2-7-16.txt"),
         "burke9": ("Burke2012_s9r23.yaml", "thermo_Burke2012_s9r23.txt"),
         # BASELINE config 4's 53-species table (gri30's 36 species cycled to 53, N2 last)
         "gri53": ("gri30.yaml", "thermo_gri53_synthetic.txt")}


def _mech(mech):
    from dfmi.mech import read_thermo_table, read_yaml_mechanism
    if mech == "gri53":
        from dfmi.synthetic import gri53_species
        sp = gri53_species(os.path.join(GOLDEN, "gri30.yaml"))
        return {"species": sp}, read_thermo_table(os.path.join(GOLDEN, MECHS[mech][1]), sp)
    ym = read_yaml_mechanism(os.path.join(GOLDEN, MECHS[mech][0]))
    return ym, read_thermo_table(os.path.join(GOLDEN, MECHS[mech][1]), ym["species"])


def _distorted_mesh(nx, ny, nz, lengths, seed=5, amp=0.15):
    """a walled hex box whose interior points are moved by up to `amp` cells at random (non-orthogonal,
    non-planar faces), written as constant/polyMesh and read back through dfmi.polymesh"""
    import tempfile
    from dfmi.polymesh import hex_polymesh, read_polymesh, write_polymesh
    P, faces, own, nei, bnd = hex_polymesh(nx, ny, nz, lengths=lengths, periodic=(False,) * 3)
    h = np.array(lengths) / np.array([nx, ny, nz])
    inner = np.all((P > 1e-12) & (P < np.array(lengths) - 1e-12), axis=1)
    P = P.copy()
    P[inner] += amp * h * np.random.default_rng(seed).uniform(-1, 1, (inner.sum(), 3))
    with tempfile.TemporaryDirectory() as d:
        write_polymesh(d, P, faces, own, nei, bnd)
        return read_polymesh(d)


def _case(nx=6, ny=5, nz=4, periodic=True, walls=None, gradings=(1.0, 1.4, 1.0), mech="es80", distorted=False,
          renumber=None, mixed=False, traversal=False, schemes=None):
    from dfmi.mesh import hex_box, FIXED_VALUE, ZERO_GRADIENT
    from dfmi.lib import Context
    from dfmi import case
    ym, t = _mech(mech)
    L = 1e-3
    if distorted:
        m = _distorted_mesh(nx, ny, nz, (2 * np.pi * L,) * 3)
    else:
        m = hex_box(nx, ny, nz, lengths=(2 * np.pi * L,) * 3, periodic=(periodic,) * 3, gradings=gradings)
    if renumber:      # the production cell order (dfmi_renumber_cells): oracle and GPU both on it
        from dfmi.renumber import renumber_mesh
        m, _ = renumber_mesh(m, renumber)
    ctx = Context(0)
    pt = case.default_patch_types(m)
    if walls:
        pt.update(walls(m))
    inert = ym["species"].index("N2")
    dt = 1e-6
    case.setup_context(ctx, m, t, inert, dt, pt, schemes=schemes)
    if traversal:     # gather kernels visit the cells in 8x8x4 bricks (dfmi_set_traversal); data order unchanged
        from dfmi.lib import renumber_cells
        ijk = np.stack(m.local_index, axis=1).astype(np.float64)
        ctx.set_traversal(renumber_cells(m.n_cells, ijk, m.owner, m.neighbour, "bricks"))
    f = case.tgv_fields(m, ym["species"], kernel_radius=1.2e-3)
    if mech == "gri53":   # every one of the 53 species present (Dirichlet-like draws)
        from dfmi.synthetic import gri53_mass_fractions
        f["Y"] = gri53_mass_fractions(m.n_cells, seed=1)
    refs = gammas = None
    if mixed:   # inletOutlet U/Y and waveTransmissive p on "right": the TGV flow crosses it both ways
        yu, _ = case.h2_air_compositions(ym["species"])
        refs = {"U": {"right": np.array([0.3, -0.1, 0.2])}, "Y": {"right": yu}}
        gammas = {"right": 1.4}
    case.init_state(ctx, m, t.S, f["T"], f["p"], f["U"], f["Y"], refs=refs, gammas=gammas)
    ctx.call("pre_time_step")
    rng = np.random.default_rng(7)
    # perturb old-time fields so ddt/ddtCorr terms are exercised
    st = case.pull_state(ctx, m, t.S)
    st["rho_old"] = st["rho"] * (1 + 1e-3 * rng.standard_normal(m.n_cells))
    st["U_old"] = st["U"] * (1 + 1e-2 * rng.standard_normal((3, m.n_cells)))
    st["phi_old"] = st["phi"] * (1 + 1e-2 * rng.standard_normal(m.n_faces))
    st["K_old"] = st["K"] * (1 + 1e-2 * rng.standard_normal(m.n_cells))
    st["p_old"] = st["p"] * (1 + 1e-4 * rng.standard_normal(m.n_cells))
    st["RR"] = 1e2 * rng.standard_normal((t.S, m.n_cells))
    st["dpdt"] = 1e3 * rng.standard_normal(m.n_cells)
    case.push_state(ctx, st)
    return ctx, m, t, st, pt, inert, dt


def _oracle(m, t, st, pt, inert, dt):
    import oracle as O
    return O.Oracle(m, t, {k: v.copy() for k, v in st.items()}, pt, inert, 1.0 / dt)


# es80 / burke9: register-resident species templates; "-generic": the same cases through the
# species-chunked kernels (option fv.species_generic) that large mechanisms run; gri53: 53 species
# (BASELINE config 4) -- every variant bitwise against the same oracle
@pytest.fixture(scope="module", params=["es80", "burke9", "walls", "distorted", "burke9-generic", "walls-generic",
                                        "gri53", "gri53-walls", "burke9-morton", "burke9-bricks", "distorted-rcm", "walls-csr",
                                        "mixed", "mixed-generic", "walls-trav"])
def periodic(request):
    from dfmi import lib
    generic = request.param.endswith("-generic")
    if generic:
        lib.DEFAULT_OPTIONS["fv.species_generic"] = 1
        request.addfinalizer(lambda: lib.DEFAULT_OPTIONS.pop("fv.species_generic", None))
    if request.param.endswith("-csr"):     # face loops by the CSR walk instead of the gather rows
        lib.DEFAULT_OPTIONS["fv.csr_walk"] = 1
        request.addfinalizer(lambda: lib.DEFAULT_OPTIONS.pop("fv.csr_walk", None))
    traversal = request.param.endswith("-trav")
    param = request.param.replace("-generic", "").replace("-csr", "").replace("-trav", "")
    renumber = None
    for meth in ("morton", "bricks", "rcm"):
        if param.endswith("-" + meth):
            renumber, param = meth, param[: -len(meth) - 1]
    mech = "gri53" if param.startswith("gri53") else "burke9"
    if param in ("walls", "distorted", "gri53-walls", "mixed"):   # zeroGradient walls (+ fixedValue T/Y/U on two sides)
        from dfmi.mesh import FIXED_VALUE, FIXED_ENERGY, GRADIENT_ENERGY, INLET_OUTLET, WAVE_TRANSMISSIVE
        mixed = param == "mixed"

        def walls(m):
            fv = {}
            names = ("left",) if mixed else ("left", "right")
            fixed = [i for i, p in enumerate(m.patches) if p.name in names]
            for f in ("U", "T", "Y"):
                t = m.patch_types(0).copy()
                t[fixed] = FIXED_VALUE
                fv[f] = t
            # he follows T (OpenFOAM heBoundaryTypes): fixedEnergy where T is fixed, gradientEnergy elsewhere
            t = m.patch_types(GRADIENT_ENERGY).copy()
            t[fixed] = FIXED_ENERGY
            fv["he"] = t
            if mixed:   # an open outlet: the mixed conditions of the reference's own cases (0/p, 0/U)
                out = [i for i, p in enumerate(m.patches) if p.name == "right"]
                fv["U"][out] = INLET_OUTLET
                fv["Y"][out] = INLET_OUTLET
                fv["p"] = m.patch_types(0).copy()
                fv["p"][out] = WAVE_TRANSMISSIVE
            return fv
        # "distorted": the same walls on a non-orthogonal mesh read from constant/polyMesh files
        return _case(periodic=False, walls=walls, mech=mech, distorted=param == "distorted", renumber=renumber,
                     mixed=mixed, traversal=traversal, nx=16 if traversal else 6,
                     ny=12 if traversal else 5, nz=8 if traversal else 4)
    return _case(mech=param, renumber=renumber, nx=16 if renumber else 6, ny=8 if renumber else 5,
                 nz=4 if renumber else 4)


def _cmp_matrix(ctx, eqn, o, parts, B, nsys=1):
    out = {}
    for part in parts:
        ref = o[part]
        got = ctx.get_matrix(eqn, part, ref.size)
        out[part] = (ulp_diff(got, ref), rel_err(got, ref))
    return out


def test_rho_eqn_bitwise(periodic):
    ctx, m, t, st, pt, inert, dt = periodic
    o = _oracle(m, t, st, pt, inert, dt)
    o.rho_eqn()
    ctx.assemble("rho")
    rho = ctx.get_field("rho", (m.n_cells,))
    assert ulp_diff(rho, o["rho"]) == 0
    assert ulp_diff(ctx.get_field("boundary_rho", (m.n_boundary_slots,)), o["boundary_rho"]) == 0
    from dfmi import case
    case.push_state(ctx, st)


def test_u_eqn_assembly_bitwise(periodic):
    ctx, m, t, st, pt, inert, dt = periodic
    o = _oracle(m, t, st, pt, inert, dt)
    ref = o.u_assemble()
    ctx.assemble("U")
    res = _cmp_matrix(ctx, "U", ref, ["lower", "upper", "diag", "source", "source_solve", "internal_coeffs",
                                      "boundary_coeffs"], m.n_boundary_slots)
    bad = {k: v for k, v in res.items() if v[0] != 0}
    assert not bad, bad
    assert ulp_diff(ctx.get_field("rAU", (m.n_cells,)), o["rAU"]) == 0


def test_hbya_bitwise(periodic):
    ctx, m, t, st, pt, inert, dt = periodic
    o = _oracle(m, t, st, pt, inert, dt)
    o.u_assemble()
    o.u_hbya()
    ctx.assemble("U")
    ctx.assemble("HbyA")
    assert ulp_diff(ctx.get_field("HbyA", (3, m.n_cells)), o["HbyA"]) == 0
    assert ulp_diff(ctx.get_field("boundary_HbyA", (3, m.n_boundary_slots)), o["boundary_HbyA"]) == 0


def test_p_eqn_assembly_bitwise(periodic):
    ctx, m, t, st, pt, inert, dt = periodic
    o = _oracle(m, t, st, pt, inert, dt)
    o.u_assemble(); o.u_hbya()
    ref = o.p_assemble()
    ctx.assemble("U"); ctx.assemble("HbyA"); ctx.assemble("p")
    res = _cmp_matrix(ctx, "p", ref, ["lower", "upper", "diag", "source", "internal_coeffs", "boundary_coeffs"],
                      m.n_boundary_slots)
    bad = {k: v for k, v in res.items() if v[0] != 0}
    assert not bad, bad
    assert ulp_diff(ctx.get_field("phiHbyA", (m.n_faces,)), ref["phiHbyA"]) == 0
    assert ulp_diff(ctx.get_field("rhorAUf", (m.n_faces,)), ref["rhorAUf"]) == 0
    vf = ctx.get_field("boundary_p_vf", (m.n_boundary_slots,))     # waveTransmissive valueFraction
    assert ulp_diff(vf, o["boundary_p_vf"]) == 0


def test_y_eqn_assembly_bitwise(periodic):
    ctx, m, t, st, pt, inert, dt = periodic
    o = _oracle(m, t, st, pt, inert, dt)
    o.y_prep()
    ref = o.y_assemble()
    ctx.assemble("Y")
    for name in ("sumYDiffError", "hDiffCorrFlux"):
        assert ulp_diff(ctx.get_field(name, (3, m.n_cells)), o[name]) == 0, name
    assert ulp_diff(ctx.get_field("diffAlphaD", (m.n_cells,)), o["diffAlphaD"]) == 0
    assert ulp_diff(ctx.get_field("phiUc", (m.n_faces,)), ref["phiUc"]) == 0
    res = _cmp_matrix(ctx, "Y", ref, ["lower", "upper", "diag", "source", "internal_coeffs", "boundary_coeffs"],
                      m.n_boundary_slots)
    bad = {k: v for k, v in res.items() if v[0] != 0}
    assert not bad, bad


def _ell_width(m):
    """coupling entries per solver row: internal faces + coupled boundary slots of the busiest cell"""
    n = np.bincount(m.owner, minlength=m.n_cells) + np.bincount(m.neighbour, minlength=m.n_cells)
    for p in m.patches:
        if p.kind in ("cyclic", "processor", "processorCyclic"):
            n = n + np.bincount(p.face_cells, minlength=m.n_cells)
    return int(n.max())


def test_y_ell_rows_bitwise(periodic):
    """The production YEqn kernel (assembly written straight into the BiCGStab rows) equals the LDU
    assembly folded by the generic gather (the ldu_to_csr + addBoundaryDiag/Source role), bit for bit."""
    ctx, m, t, st, pt, inert, dt = periodic
    W = _ell_width(m)
    n = t.S - 1
    ctx.assemble("Y_ell")
    got = {p: ctx.get_solver_rows("Y", p, n * (W if p == "val" else 1) * m.n_cells) for p in ("val", "dS", "rhs")}
    ctx.assemble("Y_ell_ref")
    for p in ("val", "dS", "rhs"):
        ref = ctx.get_solver_rows("Y", p, got[p].size)
        assert ulp_diff(got[p], ref) == 0, p
        assert np.abs(ref).max() > 0, p


def test_e_eqn_assembly_bitwise(periodic):
    ctx, m, t, st, pt, inert, dt = periodic
    # species on gradientEnergy walls off their cell values, so the energy gradient is non-trivial
    from dfmi import case
    from dfmi.mesh import GRADIENT_ENERGY
    bY = st["boundary_Y"].copy()
    slot_type = np.repeat(np.asarray(pt["he"]), [p.slots for p in m.patches])
    ge = slot_type == GRADIENT_ENERGY
    bY[:, ge] *= 1.0 + 1e-2 * np.random.default_rng(3).standard_normal((t.S, int(ge.sum())))
    ctx.set_field("boundary_Y", bY)
    st2 = dict(st, boundary_Y=bY)
    o = _oracle(m, t, st2, pt, inert, dt)
    o.y_prep()
    o.energy_gradient()
    o.correct_bc("he", "he", 1)
    ref = o.e_assemble()
    ctx.assemble("Y")
    ctx.assemble("E")
    res = _cmp_matrix(ctx, "E", ref, ["lower", "upper", "diag", "source", "internal_coeffs", "boundary_coeffs"],
                      m.n_boundary_slots)
    bad = {k: v for k, v in res.items() if v[0] != 0}
    assert not bad, bad
    assert ulp_diff(ctx.get_field("boundary_heGradient", (m.n_boundary_slots,)), o["boundary_heGradient"]) == 0
    if ge.any():
        assert np.abs(o["boundary_heGradient"][ge]).max() > 0
    case.push_state(ctx, st)


def test_thermo_correct(periodic):
    ctx, m, t, st, pt, inert, dt = periodic
    from dfmi import case
    case.push_state(ctx, st)
    o = _oracle(m, t, st, pt, inert, dt)
    # move he away from the stored T so the Newton solve does work
    he = st["he"] * 1.01
    o.set("he", he); ctx.set_field("he", he)
    bhe = st["boundary_he"] * 1.01
    o.set("boundary_he", bhe); ctx.set_field("boundary_he", bhe)
    o.thermo_correct(False)
    ctx.call("thermo_correct")
    for n in ("T", "psi", "rho", "mu", "alpha"):
        assert rel_err(ctx.get_field(n, (m.n_cells,)), o[n]) < 1e-12, n
        assert rel_err(ctx.get_field("boundary_" + n, (m.n_boundary_slots,)), o["boundary_" + n]) < 1e-12, n
    for n in ("rhoD", "hai"):
        assert rel_err(ctx.get_field(n, (t.S, m.n_cells)), o[n]) < 1e-12, n
        assert rel_err(ctx.get_field("boundary_" + n, (t.S, m.n_boundary_slots)), o["boundary_" + n]) < 1e-12, n
    case.push_state(ctx, st)


def test_full_outer_iteration(periodic):
    """One dfLowMachFoam outer iteration (nCorr = 2) vs the oracle with exact solves."""
    ctx, m, t, st, pt, inert, dt = periodic
    from dfmi import case
    case.push_state(ctx, st)
    for e in ("U", "Y", "E"):
        ctx.set_solver(e, 200, 1e-15, 1e-300)
    ctx.set_solver("p", 2000, 1e-15, 1e-300)
    o = _oracle(m, t, st, pt, inert, dt)
    o.time_step(2)
    ctx.time_step(2)
    tol = {"T": 1e-10, "p": 1e-11, "rho": 1e-10, "he": 1e-10}
    for n, tl in tol.items():
        got = ctx.get_field(n, (m.n_cells,))
        assert rel_err(got, o[n]) < tl, (n, rel_err(got, o[n]))
    U = ctx.get_field("U", (3, m.n_cells))
    assert rel_err(U, o["U"]) < 1e-9
    Y = ctx.get_field("Y", (t.S, m.n_cells))
    assert rel_err(Y, o["Y"]) < 1e-9            # per species (trace species included)
    phi = ctx.get_field("phi", (m.n_faces,))
    assert rel_err(phi, o["phi"]) < 1e-9
    B = m.n_boundary_slots
    for n, shp in (("boundary_U", (3, B)), ("boundary_Y", (t.S, B)), ("boundary_p", (B,)), ("boundary_phi", (B,))):
        assert rel_err(ctx.get_field(n, shp), o[n]) < 1e-9, n
    from dfmi.mesh import INLET_OUTLET
    io = np.repeat(np.asarray(pt["U"]) == INLET_OUTLET, [p.slots for p in m.patches])
    if io.any():   # inletOutlet switched per slot on the flux sign: inflow -> inletValue, outflow -> cell
        bphi = ctx.get_field("boundary_phi", (B,))
        assert (io & (bphi < 0)).any() and (io & (bphi >= 0)).any()
    for e in ("U", "Y", "E"):
        ctx.set_solver(e, 20, 1e-5)
    ctx.set_solver("p", 1000, 1e-5)


@pytest.mark.parametrize("prec", ["f32", "f64"])
@pytest.mark.parametrize("coarsest", ["16", "4096"])
def test_amg_pcg_full_step(coarsest, prec, monkeypatch):
    """AMG-preconditioned p solves (multi-level hierarchy forced on a small mesh) reach the oracle's
    exact solution with the V-cycle in fp32 (default) or fp64 -- the preconditioner's precision
    changes the iteration count, not the attainable accuracy; AMG needs fewer iterations than Jacobi."""
    from dfmi import lib
    monkeypatch.setitem(lib.DEFAULT_OPTIONS, "amg.coarsest_size", int(coarsest))
    monkeypatch.setitem(lib.DEFAULT_OPTIONS, "amg.precision", 64 if prec == "f64" else 32)
    ctx, m, t, st, pt, inert, dt = _case(nx=16, ny=12, nz=8, mech="burke9")
    for e in ("U", "Y", "E"):
        ctx.set_solver(e, 300, 1e-15, 1e-300)
    ctx.set_solver("p", 3000, 1e-14, 1e-300)
    o = _oracle(m, t, st, pt, inert, dt)
    o.time_step(2)
    ctx.time_step(2)
    it_amg = ctx.solver_stats("p")[0]
    for n, tl in {"T": 1e-10, "p": 1e-11, "rho": 1e-10}.items():
        got = ctx.get_field(n, (m.n_cells,))
        assert rel_err(got, o[n]) < tl, (n, rel_err(got, o[n]))
    assert rel_err(ctx.get_field("U", (3, m.n_cells)), o["U"]) < 1e-9
    from dfmi import case
    case.push_state(ctx, st)
    ctx.set_preconditioner("p", "jacobi")
    ctx.time_step(2)
    it_jac = ctx.solver_stats("p")[0]
    assert it_amg < it_jac, (it_amg, it_jac)


@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_small_solves_match_batched_path(prec, monkeypatch):
    """Systems of <= 4096 cells on one rank are solved in one workgroup per system (k_bcg_small /
    k_pcg_small with the V-cycle inside); the batched multi-launch path (option solver.small = 0) is what
    larger meshes run. Same formulas and stopping tests, reductions grouped differently: the two reach
    the same solution (tight tolerances) and the same iteration counts (within one) at production
    tolerances."""
    from dfmi import case, lib
    monkeypatch.setitem(lib.DEFAULT_OPTIONS, "amg.precision", 64 if prec == "f64" else 32)
    monkeypatch.setitem(lib.DEFAULT_OPTIONS, "amg.coarsest_size", 64)      # a multi-level hierarchy on this mesh
    res = {}
    for small in ("1", "0"):
        # solver.small decides the solver rows' layout when they are built (the first solve): one context per arm
        monkeypatch.setitem(lib.DEFAULT_OPTIONS, "solver.small", int(small))
        ctx, m, t, st, pt, inert, dt = _case(nx=16, ny=12, nz=8, mech="burke9")
        out = {}
        for tight in (True, False):
            case.push_state(ctx, st)
            if tight:
                for e in ("U", "Y", "E"):
                    ctx.set_solver(e, 300, 1e-15, 1e-300)
                ctx.set_solver("p", 3000, 1e-14, 1e-300)
            else:
                for e in ("U", "Y", "E"):
                    ctx.set_solver(e, 20, 1e-5)
                ctx.set_solver("p", 1000, 1e-5)
            ctx.time_step(2)
            out[tight] = ({n: ctx.get_field(n, (m.n_cells,)) for n in ("T", "p", "rho")} |
                          {"U": ctx.get_field("U", (3, m.n_cells)), "Y": ctx.get_field("Y", (t.S, m.n_cells))},
                          {e: ctx.solver_stats(e)[0] for e in ("U", "Y", "E", "p")})
        res[small] = out
    for n in ("T", "p", "rho", "U", "Y"):
        e = rel_err(res["1"][True][0][n], res["0"][True][0][n])
        assert e < 1e-10, (n, e)
    for e in ("U", "Y", "E", "p"):
        assert abs(res["1"][False][1][e] - res["0"][False][1][e]) <= 1, (e, res["1"][False][1], res["0"][False][1])
    case.push_state(ctx, st)
