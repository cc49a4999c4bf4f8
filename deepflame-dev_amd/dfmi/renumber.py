"""Host-side mesh renumbering (renumberMesh's role): applies the library's cell order
(dfmi_renumber_cells: Morton bricks by default) and the re-sorted faces (dfmi_renumber_faces) to a
:class:`dfmi.mesh.Mesh`, and carries cell / face fields between the two numberings.

A decomposed mesh keeps rank-blocked global cell ids (offset + local id), so a processor patch's
procCols are mapped through the PEER's permutation. `renumber_mesh` alone handles equal blocks (every
rank of a `hex_box` decomposition has the same block shape, hence the same permutation) and refuses
anything else; `renumber_decomposed` renumbers all ranks of an arbitrary decomposition (unequal cell
counts, cumulative offsets -- dfmi.partition's output) and maps every procCol through its own peer's
permutation, the peer found from the rank offsets.
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
    C = m.n_cells
    for p in m.patches:
        q = copy.copy(p)
        q.face_cells = o2n[p.face_cells].astype(np.int32)
        if p.nbr_cells_global is not None:
            # peer = g // C presumes equal blocks at offsets rank * C: refuse meshes that cannot be that
            if m.global_offset % C != 0 or (m.n_total_cells or C) % C != 0:
                raise ValueError("renumber_mesh: rank blocks of unequal size (offset %d, %d cells, %d in total); "
                                 "use renumber_decomposed" % (m.global_offset, C, m.n_total_cells))
            g = np.asarray(p.nbr_cells_global, dtype=np.int64)
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


def renumber_decomposed(meshes: list, method: str = "bricks"):
    """Renumber every rank's mesh of a decomposition ([rank] -> Mesh with global_offset and procCols in
    rank-blocked global ids, any block sizes): -> ([renumbered mesh], [Renumbering]). Each procCol g is
    split by the rank offsets (searchsorted) into (peer, local id) and mapped through that peer's own
    cell permutation."""
    offs = np.array([mm.global_offset for mm in meshes] + [meshes[-1].global_offset + meshes[-1].n_cells],
                    dtype=np.int64)
    if np.any(np.diff(offs) != np.array([mm.n_cells for mm in meshes])):
        raise ValueError("renumber_decomposed: meshes must be in rank order with contiguous global offsets")
    out, rens = [], []
    for mm in meshes:
        # each rank alone (procCols fixed below): detach them so renumber_mesh's equal-block mapping is skipped
        bare = copy.copy(mm)
        bare.patches = [copy.copy(p) for p in mm.patches]
        for p in bare.patches:
            p.nbr_cells_global = None
        r2, r = renumber_mesh(bare, method)
        out.append(r2)
        rens.append(r)
    for mm, r2 in zip(meshes, out):
        for p_old, p_new in zip(mm.patches, r2.patches):
            if p_old.nbr_cells_global is None:
                continue
            g = np.asarray(p_old.nbr_cells_global, dtype=np.int64)
            peer = np.searchsorted(offs, g, side="right") - 1
            loc = g - offs[peer]
            new_loc = np.empty_like(loc)
            for q in np.unique(peer):
                sel = peer == q
                new_loc[sel] = rens[q].cell_old_to_new[loc[sel]]
            p_new.nbr_cells_global = (offs[peer] + new_loc).astype(np.int32)
    return out, rens
