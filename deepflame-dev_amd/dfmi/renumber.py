"""Host-side mesh renumbering (renumberMesh's role): applies the library's cell order
(dfmi_renumber_cells: Morton bricks by default) and the re-sorted faces (dfmi_renumber_faces) to a
:class:`dfmi.mesh.Mesh`, and carries cell / face fields between the two numberings.

A decomposed mesh keeps rank-blocked global cell ids (offset + local id), so a processor patch's
procCols are mapped through the PEER's permutation: every rank of a `hex_box` decomposition has the
same block shape, hence the same permutation (pass `peer_perm` for anything else).
"""
from __future__ import annotations

import copy

import numpy as np

from .lib import renumber_cells, renumber_faces
from .mesh import Mesh


class Renumbering:
    def __init__(self, cell_new_to_old, face_new_to_old, face_flip):
        self.cells = np.asarray(cell_new_to_old, dtype=np.int64)
        self.faces = np.asarray(face_new_to_old, dtype=np.int64)
        self.flip = np.asarray(face_flip, dtype=bool)
        self.cell_old_to_new = np.empty_like(self.cells)
        self.cell_old_to_new[self.cells] = np.arange(self.cells.size)

    def cell_field(self, a):
        """old-numbered cell field [.., C] -> new numbering"""
        return np.ascontiguousarray(np.asarray(a)[..., self.cells])

    def cell_field_back(self, a):
        """new-numbered cell field -> old numbering"""
        return np.ascontiguousarray(np.asarray(a)[..., self.cell_old_to_new])

    def face_flux(self, a):
        """old-numbered face flux (phi-like, oriented owner -> neighbour) -> new numbering"""
        v = np.asarray(a)[..., self.faces].copy()
        v[..., self.flip[...]] *= -1.0
        return v


def renumber_mesh(m: Mesh, method: str = "bricks", peer_perm=None):
    """(renumbered mesh, Renumbering). Geometry is permuted, never recomputed."""
    # structured boxes order by their integer (i, j, k) -- the same permutation on every rank block of
    # a decomposition, whatever the grading; other meshes by their cell centres
    if method == "bricks" and not hasattr(m, "local_index"):
        method = "morton"             # unstructured: no (i, j, k) -- Z-order of the centres
    key = np.stack(m.local_index, axis=1).astype(np.float64) if hasattr(m, "local_index") else m.cell_centres
    perm = renumber_cells(m.n_cells, key, m.owner, m.neighbour, method)
    fo, no, nn, fl = renumber_faces(m.n_cells, m.owner, m.neighbour, perm)
    r = Renumbering(perm, fo, fl)
    sgn = np.where(fl, -1.0, 1.0)
    w = m.weight[fo]
    r2 = copy.copy(m)
    r2.owner = no.astype(np.int32)
    r2.neighbour = nn.astype(np.int32)
    r2.sf = np.ascontiguousarray(m.sf[fo] * sgn[:, None])
    r2.mag_sf = np.ascontiguousarray(m.mag_sf[fo])
    r2.weight = np.ascontiguousarray(np.where(fl, 1.0 - w, w))
    r2.delta_coeffs = np.ascontiguousarray(m.delta_coeffs[fo])
    r2.mesh_distance = np.ascontiguousarray(m.mesh_distance[fo] * sgn[:, None])
    r2.volume = np.ascontiguousarray(m.volume[perm])
    r2.cell_centres = np.ascontiguousarray(m.cell_centres[perm])
    o2n = r.cell_old_to_new
    pp = o2n if peer_perm is None else peer_perm
    r2.patches = []
    for p in m.patches:
        q = copy.copy(p)
        q.face_cells = o2n[p.face_cells].astype(np.int32)
        if p.nbr_cells_global is not None:
            g = np.asarray(p.nbr_cells_global, dtype=np.int64)
            C = m.n_cells
            peer, loc = g // C, g % C
            q.nbr_cells_global = (peer * C + pp[loc]).astype(np.int32)
        r2.patches.append(q)
    if hasattr(m, "local_index"):
        r2.local_index = tuple(np.asarray(a)[perm] for a in m.local_index)
    for k in ("block", "block_dims"):
        if hasattr(m, k):
            setattr(r2, k, getattr(m, k))
    r2.renumbering = r
    return r2, r
