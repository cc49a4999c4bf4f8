"""Domain decomposition of arbitrary meshes (dfmi/partition.py; the decomposePar + scotch role,
reference test/Tu500K-Phi1/system/decomposeParDict:20): partitioners, per-rank meshes in the ABI's
processor-patch conventions, processor* directory round trip, and the host halo statement
(dfmi/decomp.py) over them reproducing the serial neighbour values."""
import os
import tempfile

import numpy as np
import pytest

from conftest import ROOT


def _polymesh(nx=8, ny=6, nz=5, periodic=(True, False, True), distort=0.15, seed=3):
    from dfmi.polymesh import hex_polymesh, write_polymesh, read_polymesh
    L = 2 * np.pi * 1e-3
    P, faces, own, nei, bnd = hex_polymesh(nx, ny, nz, lengths=(L,) * 3, periodic=periodic, gradings=(1.0, 1.3, 1.0))
    h = L / np.array([nx, ny, nz])
    inner = np.all((P > 1e-12) & (P < L - 1e-12), axis=1)
    P = P.copy()
    P[inner] += distort * h * np.random.default_rng(seed).uniform(-1, 1, (inner.sum(), 3))
    d = tempfile.mkdtemp()
    write_polymesh(os.path.join(d, "constant", "polyMesh"), P, faces, own, nei, bnd)
    return d, (P, faces, own, nei, bnd), read_polymesh(os.path.join(d, "constant", "polyMesh"))


@pytest.mark.parametrize("method", ["rcb", "graph"])
@pytest.mark.parametrize("n", [2, 3, 4, 8])
def test_partition_balanced_and_complete(method, n):
    from dfmi.partition import partition_cells, edge_cut
    _, _, m = _polymesh()
    part = partition_cells(m, n, method)
    cnt = np.bincount(part, minlength=n)
    assert part.min() == 0 and part.max() == n - 1 and cnt.sum() == m.n_cells
    assert cnt.max() - cnt.min() <= max(4, 0.05 * m.n_cells / n)   # refinement: +-1 cell per bisection level
    # a useful cut: well below a random assignment's
    rnd = np.random.default_rng(0).integers(0, n, m.n_cells)
    assert edge_cut(m, part) < 0.5 * edge_cut(m, rnd)


def _check_decomposition(m, subs, part):
    R = len(subs)
    assert sum(s.n_cells for s in subs) == m.n_cells
    gid_of = np.zeros(m.n_cells, np.int64)
    for s in subs:
        gid_of[s.cell_map] = s.global_offset + np.arange(s.n_cells)
        assert np.all(np.diff(s.cell_map) > 0)            # original relative order
        o, n = s.owner.astype(np.int64), s.neighbour.astype(np.int64)
        assert np.all(o < n) and np.all(np.diff(o * s.n_cells + n) > 0)   # upper-triangular
    n_int = sum(s.n_faces for s in subs)
    proc = {}
    for s in subs:
        for p in s.patches:
            if p.kind in ("processor", "processorCyclic"):
                proc[(s.rank, p.peer_rank, getattr(p, "refer_patch", None))] = (s, p)
    n_proc_faces = sum(p.size for (_, p) in proc.values() if p.kind == "processor")
    assert n_int + n_proc_faces // 2 == m.n_faces       # every serial internal face exactly once
    for (r, q, ref), (s, p) in proc.items():
        if p.kind != "processor":
            continue
        t, pq = proc[(q, r, None)]
        assert pq.size == p.size
        mine = s.global_offset + p.face_cells
        assert np.array_equal(p.nbr_cells_global, t.global_offset + pq.face_cells)   # matching face order
        assert np.array_equal(pq.nbr_cells_global, mine)
        assert np.allclose(p.sf, -pq.sf, rtol=0, atol=1e-15 * np.abs(p.sf).max())
        assert np.allclose(p.weight + pq.weight, 1.0, rtol=0, atol=1e-12)
        assert np.allclose(p.delta_coeffs, pq.delta_coeffs, rtol=1e-12)
    for (r, q, ref), (s, p) in proc.items():
        if p.kind != "processorCyclic":
            continue
        partner = [k for k in proc if k[0] == q and k[1] == r and k[2] is not None and k[2] != ref or
                   (k[0] == q and k[1] == r and k[2] == ref and q == r)]
        assert partner, (r, q, ref)


@pytest.mark.parametrize("method,n", [("rcb", 2), ("rcb", 4), ("graph", 3), ("graph", 8)])
def test_decompose_structure(method, n):
    from dfmi.partition import partition_cells, decompose
    _, _, m = _polymesh()
    part = partition_cells(m, n, method)
    subs = decompose(m, part)
    _check_decomposition(m, subs, part)


def test_processor_directories_round_trip():
    from dfmi.partition import partition_cells, decompose, write_decomposed, read_decomposed
    d, raw, m = _polymesh()
    part = partition_cells(m, 4, "graph")
    write_decomposed(d, *raw, part)
    got = read_decomposed(d)
    ref = decompose(m, part)
    assert len(got) == len(ref) == 4
    for g, r in zip(got, ref):
        assert g.n_cells == r.n_cells and np.array_equal(g.cell_map, r.cell_map)
        assert np.array_equal(g.owner, r.owner) and np.array_equal(g.neighbour, r.neighbour)
        for a in ("sf", "mag_sf", "weight", "delta_coeffs", "volume", "cell_centres"):
            x, y = getattr(g, a), getattr(r, a)
            assert np.allclose(x, y, rtol=1e-11, atol=1e-14 * np.abs(y).max()), a
        assert [p.name for p in g.patches] == [p.name for p in r.patches]
        for pg, pr in zip(g.patches, r.patches):
            assert pg.kind == pr.kind and np.array_equal(pg.face_cells, pr.face_cells), pg.name
            assert np.allclose(pg.weight, pr.weight, rtol=1e-11), pg.name
            assert np.allclose(pg.delta_coeffs, pr.delta_coeffs, rtol=1e-11), pg.name
            if pg.kind in ("processor", "processorCyclic"):
                assert np.array_equal(pg.nbr_cells_global, pr.nbr_cells_global), pg.name


def test_halo_plan_reproduces_serial_neighbours():
    """dfmi/decomp.py's exchange over the decomposed meshes delivers, on every processor slot, the value
    of the serial cell across the face"""
    from dfmi.partition import partition_cells, decompose
    from dfmi.decomp import halo_plan, exchange_numpy
    _, _, m = _polymesh()
    part = partition_cells(m, 4, "rcb")
    subs = decompose(m, part)
    field = np.random.default_rng(1).standard_normal(m.n_cells)
    plans = [halo_plan(s) for s in subs]
    cells = [field[s.cell_map][None, :] for s in subs]
    bnd = [np.zeros((1, s.n_boundary_slots)) for s in subs]
    exchange_numpy(plans, cells, bnd)
    bnd = [b[0] for b in bnd]
    gid_to_serial = np.zeros(m.n_cells, np.int64)
    for s in subs:
        gid_to_serial[s.global_offset + np.arange(s.n_cells)] = s.cell_map
    for s, b in zip(subs, bnd):
        off = 0
        for p in s.patches:
            if p.kind in ("processor", "processorCyclic"):
                assert np.array_equal(b[off:off + p.size], field[gid_to_serial[p.nbr_cells_global]]), p.name
            off += p.slots
