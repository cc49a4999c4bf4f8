"""Domain decomposition of arbitrary meshes: the roles of decomposePar + scotch
(reference test/Tu500K-Phi1/system/decomposeParDict:20 `method scotch`) and of the processor*
directories OpenFOAM writes and the reference's decomposed runs read.

* partition_cells(m, n, method): cell -> rank. "rcb" = recursive coordinate bisection of the cell
  centres (split along the longest extent, part sizes proportional for any n); "graph" = recursive
  graph bisection on the face graph (pseudo-peripheral BFS level sets, then greedy boundary refinement
  that lowers the edge cut at fixed balance) -- no geometry needed.
* decompose(m, part): the per-rank Mesh objects decomposePar would produce, in the conventions the
  ABI expects (createGPUSolver.H:103-351): cells of a rank in their original relative order (so the
  upper-triangular face order survives), internal faces in original order, every physical patch on
  every rank (possibly empty), then one `processor` patch per neighbouring rank (faces in original face
  order, oriented outward from the rank's cells: the neighbour side sees -Sf and 1 - w), and one
  `processorCyclic` patch per (neighbour rank, cyclic patch) for cyclic pairs that straddle ranks.
  Global cell ids are rank-blocked (OpenFOAM globalIndex): procCols = offset[peer] + peer-local id.
  Geometry is copied from the serial mesh, so the decomposed operators equal the serial ones.
* write_decomposed / read_decomposed: processor<N>/constant/polyMesh directories (points, faces,
  owner, neighbour, boundary with processor / processorCyclic entries carrying myProcNo, neighbProcNo,
  referPatch; cellProcAddressing), read back into the same Mesh objects (geometry recomputed from the
  points, coupled-patch weights from both sides' face-normal distances).
"""
from __future__ import annotations

import os

import numpy as np

from .mesh import Mesh, Patch
from . import polymesh as pm


# ------------------------------------------------------------------ partitioners
def _adjacency(m: Mesh):
    """CSR of the cell graph: internal faces plus cyclic couplings"""
    a = [m.owner, m.neighbour]
    b = [m.neighbour, m.owner]
    for p in m.patches:
        if p.kind == "cyclic" and p.size:
            q = m.patches[p.neighbour_patch]
            a.append(p.face_cells); b.append(q.face_cells)
    a = np.concatenate(a).astype(np.int64)
    b = np.concatenate(b).astype(np.int64)
    keep = a != b
    a, b = a[keep], b[keep]
    order = np.lexsort((b, a))
    a, b = a[order], b[order]
    start = np.zeros(m.n_cells + 1, np.int64)
    np.add.at(start, a + 1, 1)
    return np.cumsum(start), b


def _rcb(cc, idx, nparts, first, out):
    if nparts == 1:
        out[idx] = first
        return
    k0 = nparts // 2
    n0 = int(round(idx.size * k0 / nparts))
    pts = cc[idx]
    ax = int(np.argmax(pts.max(axis=0) - pts.min(axis=0)))
    order = np.lexsort((idx, pts[:, ax]))     # ties by cell index: deterministic
    _rcb(cc, idx[order[:n0]], k0, first, out)
    _rcb(cc, idx[order[n0:]], nparts - k0, first + k0, out)


def _bfs_order(start, adj, cells, mask, seed):
    """BFS order of the sub-graph `mask` from seed; unreached components appended (each BFS'd)"""
    seen = np.zeros(mask.size, bool)
    order = []
    pending = [seed] + [int(c) for c in cells]
    for s in pending:
        if seen[s]:
            continue
        seen[s] = True
        frontier = [s]
        while frontier:
            order.extend(frontier)
            nxt = []
            for c in frontier:
                for j in adj[start[c]:start[c + 1]]:
                    if mask[j] and not seen[j]:
                        seen[j] = True
                        nxt.append(int(j))
            frontier = nxt
    return np.array(order, np.int64)


def _refine(start, adj, part, a, b, target_a, passes=4):
    """greedy boundary refinement between parts a and b: move a cell when it lowers the edge cut and
    keeps part a within 1 % (and one cell) of its target size"""
    tol = max(1, int(0.01 * target_a))
    for _ in range(passes):
        moved = 0
        cells = np.flatnonzero((part == a) | (part == b))
        na = int((part == a).sum())
        for c in cells:
            pc = part[c]
            other = b if pc == a else a
            nb = adj[start[c]:start[c + 1]]
            gain = int((part[nb] == other).sum()) - int((part[nb] == pc).sum())
            if gain <= 0:
                continue
            new_na = na - 1 if pc == a else na + 1
            if abs(new_na - target_a) > tol:
                continue
            part[c] = other
            na = new_na
            moved += 1
        if not moved:
            break


def _rgb(start, adj, idx, nparts, first, out):
    if nparts == 1:
        out[idx] = first
        return
    k0 = nparts // 2
    n0 = int(round(idx.size * k0 / nparts))
    mask = np.zeros(out.size, bool)
    mask[idx] = True
    # pseudo-peripheral seed: the last cell of a BFS from the lowest index, twice
    seed = int(idx.min())
    for _ in range(2):
        seed = int(_bfs_order(start, adj, idx, mask, seed)[-1])
    order = _bfs_order(start, adj, idx, mask, seed)
    tmp = np.full(out.size, -1, np.int64)
    tmp[order[:n0]] = 0
    tmp[order[n0:]] = 1
    _refine(start, adj, tmp, 0, 1, n0)
    _rgb(start, adj, np.flatnonzero(tmp == 0), k0, first, out)
    _rgb(start, adj, np.flatnonzero(tmp == 1), nparts - k0, first + k0, out)


def partition_cells(m: Mesh, nparts: int, method: str = "rcb") -> np.ndarray:
    """cell -> rank for nparts ranks"""
    if nparts < 1 or nparts > m.n_cells:
        raise ValueError("bad part count")
    out = np.full(m.n_cells, -1, np.int64)
    if method == "rcb":
        _rcb(np.asarray(m.cell_centres), np.arange(m.n_cells), nparts, 0, out)
    elif method == "graph":
        start, adj = _adjacency(m)
        _rgb(start, adj, np.arange(m.n_cells), nparts, 0, out)
    else:
        raise ValueError("method must be 'rcb' or 'graph'")
    return out.astype(np.int32)


def edge_cut(m: Mesh, part: np.ndarray) -> int:
    start, adj = _adjacency(m)
    src = np.repeat(np.arange(m.n_cells), np.diff(start))
    return int((part[src] != part[adj]).sum() // 2)


# ------------------------------------------------------------------ decomposition
def decompose(m: Mesh, part: np.ndarray) -> list:
    """per-rank Meshes (see the module docstring); each carries cell_map (local -> serial cell id)"""
    part = np.asarray(part, np.int64)
    R = int(part.max()) + 1
    counts = np.bincount(part, minlength=R)
    if (counts == 0).any():
        raise ValueError("empty part")
    offset = np.concatenate([[0], np.cumsum(counts)[:-1]])
    local = np.zeros(m.n_cells, np.int64)
    for r in range(R):
        local[part == r] = np.arange(counts[r])
    po, pn = part[m.owner], part[m.neighbour]
    cut = po != pn
    out = []
    for r in range(R):
        cells = np.flatnonzero(part == r)
        fi = np.flatnonzero((po == r) & ~cut)
        patches = []
        # physical patches (every rank keeps every patch, decomposePar style); cyclic pairs split below
        cyc_keep = {}
        for pi, p in enumerate(m.patches):
            if p.kind == "cyclic":
                q = m.patches[p.neighbour_patch]
                mine = part[p.face_cells] == r
                same = part[q.face_cells] == r
                cyc_keep[pi] = np.flatnonzero(mine & same)
                sel = cyc_keep[pi]
            else:
                sel = np.flatnonzero(part[p.face_cells] == r)
            np_ = Patch(p.name, p.kind, local[p.face_cells[sel]].astype(np.int32), p.sf[sel], p.mag_sf[sel],
                        p.weight[sel], p.delta_coeffs[sel])
            np_.neighbour_patch = p.neighbour_patch
            patches.append(np_)
        # processor patches: one per neighbour rank, faces in serial face order
        peers = sorted(set(pn[(po == r) & cut].tolist()) | set(po[(pn == r) & cut].tolist()))
        for q in peers:
            f_own = np.flatnonzero((po == r) & (pn == q))
            f_nei = np.flatnonzero((pn == r) & (po == q))
            f = np.sort(np.concatenate([f_own, f_nei]))
            is_own = po[f] == r
            fc = np.where(is_own, m.owner[f], m.neighbour[f])
            oc = np.where(is_own, m.neighbour[f], m.owner[f])
            sgn = np.where(is_own, 1.0, -1.0)[:, None]
            w = np.where(is_own, m.weight[f], 1.0 - m.weight[f])
            p = Patch(f"procBoundary{r}to{q}", "processor", local[fc].astype(np.int32), m.sf[f] * sgn, m.mag_sf[f].copy(),
                      w, m.delta_coeffs[f].copy(), peer_rank=q)
            p.nbr_cells_global = (offset[q] + local[oc]).astype(np.int32)
            patches.append(p)
        # processorCyclic: cyclic pairs across ranks, one patch per (peer, cyclic patch), pair order
        for pi, p in enumerate(m.patches):
            if p.kind != "cyclic":
                continue
            q_p = m.patches[p.neighbour_patch]
            mine = np.flatnonzero((part[p.face_cells] == r) & (part[q_p.face_cells] != r))
            for q in sorted(set(part[q_p.face_cells[mine]].tolist())):
                sel = mine[part[q_p.face_cells[mine]] == q]
                pp = Patch(f"procBoundary{r}to{q}through{p.name}", "processorCyclic", local[p.face_cells[sel]].astype(np.int32),
                           p.sf[sel], p.mag_sf[sel], p.weight[sel], p.delta_coeffs[sel], peer_rank=q)
                pp.nbr_cells_global = (offset[q] + local[q_p.face_cells[sel]]).astype(np.int32)
                pp.refer_patch = p.name
                patches.append(pp)
        # cyclic partner indices refer to the same patch list (physical patches keep their indices)
        sub = Mesh(n_cells=int(counts[r]), owner=local[m.owner[fi]].astype(np.int32),
                   neighbour=local[m.neighbour[fi]].astype(np.int32), sf=m.sf[fi], mag_sf=m.mag_sf[fi],
                   weight=m.weight[fi], delta_coeffs=m.delta_coeffs[fi], volume=m.volume[cells],
                   cell_centres=m.cell_centres[cells], mesh_distance=m.mesh_distance[fi], patches=patches,
                   global_offset=int(offset[r]), n_total_cells=int(m.n_cells))
        sub.cell_map = cells
        sub.rank = r
        out.append(sub)
    return out


# ------------------------------------------------------------------ processor directories
def write_decomposed(case_dir: str, points, faces, owner, neighbour, boundary, part) -> None:
    """processor<r>/constant/polyMesh of a serial polyMesh (points, faces, owner, neighbour, boundary as
    polymesh.hex_polymesh returns them: boundary = [(name, type, nFaces, startFace, neighbourPatch)])"""
    owner = np.asarray(owner, np.int64)
    neighbour = np.asarray(neighbour, np.int64)
    part = np.asarray(part, np.int64)
    R = int(part.max()) + 1
    Fi = neighbour.size
    counts = np.bincount(part, minlength=R)
    local = np.zeros(part.size, np.int64)
    for r in range(R):
        local[part == r] = np.arange(counts[r])
    bfaces = {b[0]: np.arange(b[3], b[3] + b[2]) for b in boundary}
    btype = {b[0]: b[1] for b in boundary}
    bnbr = {b[0]: b[4] for b in boundary}
    po, pn = part[owner[:Fi]], part[neighbour]
    for r in range(R):
        flist, own_l, nei_l, bnd = [], [], [], []
        fi = np.flatnonzero((po == r) & (pn == r))
        for f in fi:
            flist.append(list(faces[f])); own_l.append(local[owner[f]]); nei_l.append(local[neighbour[f]])
        for name, t, nF, s0, nbr in boundary:
            fs = bfaces[name]
            if t == "cyclic":
                pf = bfaces[nbr]
                fs = fs[(part[owner[fs]] == r) & (part[owner[pf]] == r)]
            else:
                fs = fs[part[owner[fs]] == r]
            start = len(flist)
            for f in fs:
                flist.append(list(faces[f])); own_l.append(local[owner[f]])
            bnd.append((name, t, len(fs), start, nbr, None))
        peers = sorted(set(pn[(po == r) & (pn != r)].tolist()) | set(po[(pn == r) & (po != r)].tolist()))
        for q in peers:
            f = np.sort(np.flatnonzero(((po == r) & (pn == q)) | ((pn == r) & (po == q))))
            start = len(flist)
            for ff in f:
                if po[ff] == r:
                    flist.append(list(faces[ff])); own_l.append(local[owner[ff]])
                else:   # seen from the neighbour: reversed vertex order, outward normal
                    flist.append(list(faces[ff])[::-1]); own_l.append(local[neighbour[ff]])
            bnd.append((f"procBoundary{r}to{q}", "processor", len(f), start, None, (r, q, None)))
        for name, t, nF, s0, nbr in boundary:
            if t != "cyclic":
                continue
            fs, pf = bfaces[name], bfaces[nbr]
            mine = (part[owner[fs]] == r) & (part[owner[pf]] != r)
            for q in sorted(set(part[owner[pf[mine]]].tolist())):
                sel = fs[mine & (part[owner[pf]] == q)]
                start = len(flist)
                for ff in sel:
                    flist.append(list(faces[ff])); own_l.append(local[owner[ff]])
                bnd.append((f"procBoundary{r}to{q}through{name}", "processorCyclic", len(sel), start, None, (r, q, name)))
        # local points
        used = np.unique(np.concatenate([np.asarray(f, np.int64) for f in flist]))
        pmap = np.full(len(points), -1, np.int64)
        pmap[used] = np.arange(used.size)
        lfaces = [[int(pmap[v]) for v in f] for f in flist]
        d = os.path.join(case_dir, f"processor{r}", "constant", "polyMesh")
        pm.write_polymesh(d, np.asarray(points)[used], lfaces, np.array(own_l, np.int64), np.array(nei_l, np.int64),
                          [(b[0], b[1], b[2], b[3], b[4]) for b in bnd])
        _write_proc_entries(os.path.join(d, "boundary"), bnd)
        with open(os.path.join(d, "cellProcAddressing"), "w") as fh:
            cells = np.flatnonzero(part == r)
            fh.write(pm._hdr("labelList", "cellProcAddressing") + f"{cells.size}\n(\n")
            fh.writelines("%d\n" % c for c in cells)
            fh.write(")\n")


def _write_proc_entries(path, bnd):
    """rewrite the boundary file with the processor keywords (myProcNo, neighbProcNo, referPatch)"""
    with open(path, "w") as f:
        f.write(pm._hdr("polyBoundaryMesh", "boundary") + f"{len(bnd)}\n(\n")
        for name, t, nF, s0, nbr, proc in bnd:
            f.write(f"    {name}\n    {{\n        type            {t};\n        nFaces          {nF};\n"
                    f"        startFace       {s0};\n")
            if nbr:
                f.write(f"        neighbourPatch  {nbr};\n")
            if proc:
                f.write(f"        myProcNo        {proc[0]};\n        neighbProcNo    {proc[1]};\n")
                if proc[2]:
                    f.write(f"        referPatch      {proc[2]};\n")
            f.write("    }\n")
        f.write(")\n")


def read_decomposed(case_dir: str) -> list:
    """processor<r>/constant/polyMesh directories -> per-rank Meshes (ABI conventions as decompose())"""
    R = 0
    while os.path.isdir(os.path.join(case_dir, f"processor{R}")):
        R += 1
    if R == 0:
        raise FileNotFoundError(f"no processor* directories in {case_dir}")
    raw = []
    for r in range(R):
        d = os.path.join(case_dir, f"processor{r}", "constant", "polyMesh")
        pts = pm._read_points(os.path.join(d, "points"))
        faces = pm._read_faces(os.path.join(d, "faces"))
        owner = pm._read_labels(os.path.join(d, "owner"))
        neighbour = pm._read_labels(os.path.join(d, "neighbour"))
        bnd = pm._read_boundary(os.path.join(d, "boundary"))
        C = int(max(owner.max(), neighbour.max() if neighbour.size else 0)) + 1
        Cf, Sf = pm.face_centres_areas(pts, faces)
        cc, vol = pm.cell_centres_volumes(C, owner, neighbour, Cf, Sf)
        cpa = os.path.join(d, "cellProcAddressing")
        cmap = pm._read_labels(cpa) if os.path.exists(cpa) else None
        raw.append(dict(owner=owner, neighbour=neighbour, bnd=bnd, C=C, Cf=Cf, Sf=Sf, cc=cc, vol=vol, cmap=cmap))
    offset = np.concatenate([[0], np.cumsum([x["C"] for x in raw])[:-1]])
    total = int(sum(x["C"] for x in raw))

    def patch_geo(x, d):
        nF, s0 = int(d["nFaces"]), int(d["startFace"])
        sl = slice(s0, s0 + nF)
        fc = x["owner"][sl]
        sf = x["Sf"][sl]
        mag = np.linalg.norm(sf, axis=1)
        nfv = sf / np.maximum(mag, 1e-300)[:, None]
        delta = np.einsum("ij,ij->i", nfv, x["Cf"][sl] - x["cc"][fc])[:, None] * nfv
        return fc, sf, mag, nfv, delta, x["Cf"][sl] - x["cc"][fc]

    out = []
    for r, x in enumerate(raw):
        Fi = x["neighbour"].size
        o, n = x["owner"][:Fi], x["neighbour"]
        sfi = x["Sf"][:Fi]
        d_o = np.abs(np.einsum("ij,ij->i", sfi, x["Cf"][:Fi] - x["cc"][o]))
        d_n = np.abs(np.einsum("ij,ij->i", sfi, x["cc"][n] - x["Cf"][:Fi]))
        mdist = x["cc"][n] - x["cc"][o]
        names = [b[0] for b in x["bnd"]]
        patches = []
        for name, d in x["bnd"]:
            t = d["type"].strip()
            fc, sf, mag, nfv, delta, dfull = patch_geo(x, d)
            if t in ("processor", "processorCyclic"):
                q = int(d["neighbProcNo"])
                y = raw[q]
                qnames = [b[0] for b in y["bnd"]]
                if t == "processor":
                    qname = f"procBoundary{q}to{r}"
                else:
                    nbr_patch = _cyclic_partner(raw, r, d["referPatch"].strip())
                    qname = f"procBoundary{q}to{r}through{nbr_patch}"
                qd = y["bnd"][qnames.index(qname)][1]
                qfc, _, _, qn, qdelta, qfull = patch_geo(y, qd)
                di = np.einsum("ij,ij->i", nfv, delta)
                dni = np.einsum("ij,ij->i", qn, qdelta)
                # processorFvPatch::makeWeights (face-normal distances); delta = (Cf - C) - (Cf' - C')
                p = Patch(name, t, fc.astype(np.int32), sf, mag, dni / (di + dni), 1.0 / np.linalg.norm(dfull - qfull, axis=1),
                          peer_rank=q)
                p.nbr_cells_global = (offset[q] + qfc).astype(np.int32)
                if t == "processorCyclic":
                    p.refer_patch = d["referPatch"].strip()
                patches.append(p)
                continue
            kind = pm._KIND.get(t)
            if kind is None:
                raise ValueError(f"processor{r}: patch {name} type {t} not supported")
            if kind == "empty":
                patches.append(Patch(name, "empty", fc[:0].astype(np.int32), sf[:0], mag[:0], np.ones(0), np.ones(0)))
            elif kind == "cyclic":
                qi = names.index(d["neighbourPatch"].strip())
                _, _, _, qn, qdelta, qfull = patch_geo(x, x["bnd"][qi][1])
                di = np.einsum("ij,ij->i", nfv, delta)
                dni = np.einsum("ij,ij->i", qn, qdelta)
                p = Patch(name, "cyclic", fc.astype(np.int32), sf, mag, dni / (di + dni), 1.0 / np.linalg.norm(dfull - qfull, axis=1))
                p.neighbour_patch = qi
                patches.append(p)
            else:
                patches.append(Patch(name, "wall", fc.astype(np.int32), sf, mag, np.ones(fc.size),
                                     1.0 / np.linalg.norm(delta, axis=1)))
        sub = Mesh(n_cells=x["C"], owner=o.astype(np.int32), neighbour=n.astype(np.int32), sf=sfi,
                   mag_sf=np.linalg.norm(sfi, axis=1), weight=d_n / (d_o + d_n), delta_coeffs=1.0 / np.linalg.norm(mdist, axis=1),
                   volume=x["vol"], cell_centres=x["cc"], mesh_distance=mdist, patches=patches,
                   global_offset=int(offset[r]), n_total_cells=total)
        sub.cell_map = x["cmap"]
        sub.rank = r
        out.append(sub)
    return out


def _cyclic_partner(raw, r, name):
    for nm, d in raw[r]["bnd"]:
        if nm == name:
            return d["neighbourPatch"].strip()
    raise KeyError(name)
