"""constant/polyMesh reader (case I/O row): a hex box written in polyMesh form and read back
gives the Mesh the in-process generator builds (same addressing, geometry to rounding: the reader
recomputes it with OpenFOAM's primitiveMesh / surfaceInterpolation algorithms from the points), and the
reader's geometry stays consistent on a distorted (non-orthogonal) mesh."""
import gzip
import os
import shutil

import numpy as np
import pytest

from dfmi.mesh import hex_box
from dfmi.polymesh import (cell_centres_volumes, face_centres_areas, hex_polymesh, read_polymesh,
                           write_polymesh)

CASES = [
    dict(n=(6, 5, 4), kw=dict(lengths=(1e-2, 2e-2, 3e-2), periodic=(True, True, True), gradings=(1.0, 3.0, 0.5))),
    dict(n=(7, 3, 2), kw=dict(lengths=(1.0, 0.5, 0.25), periodic=(False, True, False), gradings=(2.0, 1.0, 1.0))),
    dict(n=(40, 1, 1), kw=dict(lengths=(0.04, 1e-3, 1e-3), periodic=(False, False, False),
                               gradings=([(0.55, 0.625, 1.0), (0.45, 0.375, 2.0)], 1.0, 1.0),
                               wall_kinds={"front": "empty", "back": "empty", "top": "empty", "down": "empty"})),
]


def _close(a, b, rtol=1e-12):
    a, b = np.asarray(a, float), np.asarray(b, float)
    assert a.shape == b.shape
    scale = max(np.abs(b).max(), 1e-300) if b.size else 1.0
    assert np.all(np.abs(a - b) <= rtol * scale + 1e-300), np.abs(a - b).max() / scale


@pytest.mark.parametrize("case", CASES, ids=["periodic-graded", "walls-cyclic-y", "flame1d"])
def test_written_hex_box_reads_back(tmp_path, case):
    n, kw = case["n"], case["kw"]
    d = str(tmp_path / "polyMesh")
    write_polymesh(d, *hex_polymesh(*n, **kw))
    m = read_polymesh(d)
    ref = hex_box(*n, **kw)
    assert m.n_cells == ref.n_cells
    np.testing.assert_array_equal(m.owner, ref.owner)
    np.testing.assert_array_equal(m.neighbour, ref.neighbour)
    for a in ("sf", "mag_sf", "weight", "delta_coeffs", "volume", "cell_centres", "mesh_distance"):
        _close(getattr(m, a), getattr(ref, a))
    assert [p.name for p in m.patches] == [p.name for p in ref.patches]
    for p, q in zip(m.patches, ref.patches):
        assert p.kind == q.kind and p.neighbour_patch == q.neighbour_patch, p.name
        np.testing.assert_array_equal(p.face_cells, q.face_cells)
        for a in ("sf", "mag_sf", "weight", "delta_coeffs"):
            _close(getattr(p, a), getattr(q, a))


def test_gzipped_files(tmp_path):
    d = str(tmp_path / "polyMesh")
    write_polymesh(d, *hex_polymesh(3, 3, 3))
    for f in ("points", "faces"):
        with open(os.path.join(d, f), "rb") as src, gzip.open(os.path.join(d, f + ".gz"), "wb") as dst:
            shutil.copyfileobj(src, dst)
        os.remove(os.path.join(d, f))
    m = read_polymesh(d)
    _close(m.volume, hex_box(3, 3, 3).volume)


def test_distorted_mesh_geometry(tmp_path):
    """interior points moved at random: every cell stays closed (sum of outward area vectors = 0), the
    pyramid volumes add up to the box, weights lie in (0, 1), and a triangle face is handled"""
    P, faces, own, nei, bnd = hex_polymesh(5, 4, 3, lengths=(1.0, 1.0, 1.0), periodic=(False, False, False))
    rng = np.random.default_rng(3)
    inner = np.all((P > 1e-9) & (P < 1 - 1e-9), axis=1)
    P = P.copy()
    P[inner] += 0.01 * rng.uniform(-1, 1, (inner.sum(), 3))
    d = str(tmp_path / "polyMesh")
    write_polymesh(d, P, faces, own, nei, bnd)
    m = read_polymesh(d)
    assert abs(m.volume.sum() - 1.0) < 1e-12
    assert np.all(m.volume > 0) and np.all((m.weight > 0) & (m.weight < 1))
    Cf, Sf = face_centres_areas(P, faces)
    C = m.n_cells
    net = np.zeros((C, 3))
    for k in range(3):
        net[:, k] = np.bincount(own, Sf[:, k], C) - np.bincount(nei, Sf[:nei.size, k], C)
    assert np.abs(net).max() < 1e-14
    cc, vol = cell_centres_volumes(C, own, nei, Cf, Sf)
    _close(vol, m.volume)
    _close(cc, m.cell_centres)
    # triangle face: centroid and half the cross product
    tri = np.array([[0.0, 0.0, 0.0], [2.0, 0.0, 0.0], [0.0, 1.0, 0.0]])
    cf, sf = face_centres_areas(tri, [np.array([0, 1, 2])])
    _close(cf[0], [2.0 / 3.0, 1.0 / 3.0, 0.0])
    _close(sf[0], [0.0, 0.0, 1.0])
