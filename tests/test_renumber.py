"""Cell renumbering (dfmi_renumber_cells / dfmi_renumber_faces, renumberMesh's role): valid
permutations, upper-triangular faces, oriented geometry, Morton bricks -- and the oracle's outer
iteration on the renumbered mesh equals the one on the original numbering (CPU, no GPU needed)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, rel_err


def _check_mesh(m):
    assert np.all(m.owner < m.neighbour)
    key = m.owner.astype(np.int64) * m.n_cells + m.neighbour
    assert np.all(np.diff(key) > 0)                                # sorted by owner, then neighbour
    d = m.cell_centres[m.neighbour] - m.cell_centres[m.owner]
    assert np.all((m.sf * d).sum(axis=1) > 0)                      # Sf points owner -> neighbour
    np.testing.assert_allclose(m.mesh_distance, d, rtol=0, atol=1e-15)


@pytest.mark.parametrize("method", ["morton", "bricks"])
def test_morton_bricks_and_faces(method):
    from dfmi.mesh import hex_box
    from dfmi.renumber import renumber_mesh
    m = hex_box(16, 16, 16)
    r2, r = renumber_mesh(m, method)
    assert sorted(r.cells.tolist()) == list(range(m.n_cells))
    assert not r.flip.any()                                       # monotone order of a structured box: no flips
    _check_mesh(r2)
    ii, jj, kk = r2.local_index
    for b in range(0, m.n_cells, 256):                            # 256 consecutive cells = one 8 x 8 x 4 brick
        ext = [np.ptp(a[b:b + 256]) + 1 for a in (ii, jj, kk)]
        assert ext == [8, 8, 4], ext
    if method == "bricks":                                        # lexicographic inside the brick
        assert np.array_equal(ii[:8], np.arange(8)) and np.all(jj[:8] == 0) and jj[8] == 1
    np.testing.assert_array_equal(r2.volume, m.volume[r.cells])
    for p, q in zip(m.patches, r2.patches):
        np.testing.assert_array_equal(r.cells[q.face_cells], p.face_cells)


@pytest.mark.parametrize("method", ["morton", "rcm"])
def test_renumber_distorted_polymesh(method):
    from dfmi.polymesh import hex_polymesh, read_polymesh, write_polymesh
    from dfmi.renumber import renumber_mesh
    import tempfile
    P, faces, own, nei, bnd = hex_polymesh(6, 5, 4, lengths=(1e-3,) * 3, periodic=(False,) * 3)
    inner = np.all((P > 1e-12) & (P < 1e-3 - 1e-12), axis=1)
    P = P.copy()
    P[inner] += 0.15 * (1e-3 / 6) * np.random.default_rng(2).uniform(-1, 1, (inner.sum(), 3))
    with tempfile.TemporaryDirectory() as d:
        write_polymesh(d, P, faces, own, nei, bnd)
        m = read_polymesh(d)
    r2, r = renumber_mesh(m, method)
    _check_mesh(r2)
    if method == "rcm":
        assert r.flip.any()                                        # the general path flips faces


def _state(m, table, species):
    import oracle as O
    from dfmi import case
    f = case.tgv_fields(m, species, kernel_radius=1.2e-3)
    C_, F, B, S = m.n_cells, m.n_faces, m.n_boundary_slots, table.S
    st = {}
    for nme in case.SCALARS:
        st[nme] = np.zeros(C_); st["boundary_" + nme] = np.zeros(B)
    for nme in case.VECTORS:
        st[nme] = np.zeros((3, C_)); st["boundary_" + nme] = np.zeros((3, B))
    for nme in case.SPECIES:
        st[nme] = np.zeros((S, C_)); st["boundary_" + nme] = np.zeros((S, B))
    for nme in case.FACES:
        st[nme] = np.zeros(F); st["boundary_" + nme] = np.zeros(B)
    for k in ("T", "p", "U", "Y"):
        st[k] = f[k].copy()
        st["boundary_" + k] = case.boundary_values(m, st[k])
    o = O.Oracle(m, table, st, case.default_patch_types(m), 0, 1e6)
    o.thermo_correct(True)
    s = {k: v.copy() for k, v in o.arr.items() if k in st}
    s["phi"], s["boundary_phi"] = case.face_flux(m, s["rho"], s["U"], s["boundary_rho"], s["boundary_U"])
    s["K"] = 0.5 * (s["U"] ** 2).sum(axis=0)
    s["boundary_K"] = 0.5 * (s["boundary_U"] ** 2).sum(axis=0)
    s["RR"] = 1e2 * np.random.default_rng(4).standard_normal((S, C_))
    return s


def test_oracle_step_invariant_under_renumbering():
    import oracle as O
    from dfmi.mesh import hex_box
    from dfmi.mech import read_thermo_table, read_yaml_mechanism
    from dfmi.renumber import renumber_mesh
    from dfmi import case
    ym = read_yaml_mechanism(os.path.join(GOLDEN, "Burke2012_s9r23.yaml"))
    t = read_thermo_table(os.path.join(GOLDEN, "thermo_Burke2012_s9r23.txt"), ym["species"])
    m = hex_box(8, 6, 4, lengths=(2 * np.pi * 1e-3,) * 3, gradings=(1.0, 1.3, 1.0))
    st = _state(m, t, ym["species"])
    inert = ym["species"].index("N2")
    r2, r = renumber_mesh(m, "morton")
    st2 = {}
    for k, v in st.items():
        if k.startswith("boundary_"):
            st2[k] = v.copy()                                     # slot order is kept
        elif v.shape[-1] == m.n_cells:
            st2[k] = r.cell_field(v)
        else:
            st2[k] = r.face_flux(v)
    a = O.Oracle(m, t, st, case.default_patch_types(m), inert, 1e6)      # (one oracle registry at a time)
    a.time_step(2)
    a = {k: v.copy() for k, v in a.arr.items()}
    b = O.Oracle(r2, t, st2, case.default_patch_types(r2), inert, 1e6)
    b.time_step(2)
    for k in ("T", "p", "rho", "he", "U", "Y"):
        assert rel_err(r.cell_field_back(b[k]), a[k]) < 1e-12, k
    assert rel_err(b["phi"], r.face_flux(a["phi"])) < 1e-12


def test_renumber_decomposed_unequal_blocks():
    """a decomposition with unequal rank sizes (RCB into 3) renumbered rank by rank: every
    procCol still names the same physical cell (its centre) after both sides' permutations; renumber_mesh
    alone refuses such a mesh instead of mis-mapping it"""
    import numpy as np
    import pytest
    from dfmi.mesh import hex_box
    from dfmi.partition import partition_cells, decompose
    from dfmi.renumber import renumber_mesh, renumber_decomposed
    mg = hex_box(7, 5, 4, periodic=(True, False, True))
    part = partition_cells(mg, 3, "rcb")
    meshes = decompose(mg, part)
    sizes = [mm.n_cells for mm in meshes]
    assert len(set(sizes)) > 1
    bad = [mm for mm in meshes if mm.global_offset % mm.n_cells or mm.n_total_cells % mm.n_cells]
    assert bad
    with pytest.raises(ValueError, match="unequal"):
        renumber_mesh(bad[0], "morton")
    new, rens = renumber_decomposed(meshes, "morton")
    offs = np.array([mm.global_offset for mm in meshes] + [mg.n_cells])
    for r, (mo, mn) in enumerate(zip(meshes, new)):
        assert np.allclose(mn.cell_centres, mo.cell_centres[rens[r].cells])
        for po, pn in zip(mo.patches, mn.patches):
            if po.nbr_cells_global is None:
                continue
            go = np.asarray(po.nbr_cells_global); gn = np.asarray(pn.nbr_cells_global)
            for a, b in zip(go, gn):
                qa = np.searchsorted(offs, a, side="right") - 1
                qb = np.searchsorted(offs, b, side="right") - 1
                assert qa == qb
                assert np.allclose(meshes[qa].cell_centres[a - offs[qa]], new[qb].cell_centres[b - offs[qb]])
            # this side's face cells follow its own permutation
            assert np.allclose(mn.cell_centres[pn.face_cells], mo.cell_centres[po.face_cells])
