"""OpenFOAM constant/polyMesh reader and writer (ASCII, optionally gzip'd): the mesh part of the case
I/O row. `read_polymesh(dir)` turns points / faces / owner / neighbour /
boundary into the same `Mesh` the rest of the host code builds from (createGPUSolver.H:103-351 reads
these arrays from OpenFOAM's fvMesh), computing the geometry the way OpenFOAM does:

  * face centres and area vectors: primitiveMesh::makeFaceCentresAndAreas (triangle fan about the
    point average; a triangle face directly);
  * cell centres and volumes: primitiveMesh::makeCellCentresAndVols (face pyramids about the average
    of the cell's face centres);
  * weights: surfaceInterpolation::makeWeights  w = |Sf.(Cn - Cf)| / (|Sf.(Cf - Co)| + |Sf.(Cn - Cf)|);
    deltaCoeffs 1 / |Cn - Co| (mesh.deltaCoeffs(), what createGPUSolver.H:338-339 passes);
  * non-coupled patches: w = 1, deltaCoeffs = 1 / |nf.(Cf - Co)| (fvPatch::delta, patch-normal);
  * cyclic (translational): w = dn / (d + dn) with d = nf.(Cf - Co) on each side
    (cyclicFvPatch::makeWeights), deltaCoeffs = 1 / |(Cf - Co) - (Cf' - Cn')| (cyclicFvPatch::delta:
    full vectors, coupledFvPatch::delta, not the patch-normal ones of fvPatch::delta).

`hex_polymesh` + `write_polymesh` write the single-block hex box of `mesh.hex_box` as polyMesh files (faces
in the same order, OpenFOAM orientation: internal normals owner -> neighbour, boundary normals outward), so
a blockMesh-generated case and the in-process generator can be checked against each other. Text
parsing only; serial meshes here -- decomposed processor* directories are written and read by
dfmi/partition.py."""
from __future__ import annotations

import gzip
import os
import re

import numpy as np

from .mesh import Mesh, Patch, _axis_nodes

_KIND = {"patch": "wall", "wall": "wall", "symmetryPlane": "wall", "symmetry": "wall", "cyclic": "cyclic",
         "empty": "empty", "wedge": "wall"}


def _read(path: str) -> str:
    for p in (path, path + ".gz"):
        if os.path.exists(p):
            return gzip.open(p, "rt").read() if p.endswith(".gz") else open(p).read()
    raise FileNotFoundError(path)


def _body(txt: str) -> str:
    """the data part after the FoamFile header (comments stripped)"""
    txt = re.sub(r"/\*.*?\*/", " ", txt, flags=re.S)
    txt = re.sub(r"//[^\n]*", " ", txt)
    h = re.search(r"FoamFile\s*\{.*?\}", txt, flags=re.S)
    return txt[h.end():] if h else txt


def _list_start(body: str):
    m = re.search(r"(\d+)\s*\(", body)
    if m is None:
        raise ValueError("no list")
    return int(m.group(1)), m.end()


def _read_labels(path: str) -> np.ndarray:
    body = _body(_read(path))
    n, s = _list_start(body)
    vals = np.array(body[s:body.index(")", s)].split(), dtype=np.int64)
    assert vals.size == n, (path, vals.size, n)
    return vals.astype(np.int32)


def _read_points(path: str) -> np.ndarray:
    body = _body(_read(path))
    n, s = _list_start(body)
    end = body.rindex(")")
    nums = np.array(body[s:end].replace("(", " ").replace(")", " ").split(), dtype=np.float64)
    assert nums.size == 3 * n, (path, nums.size, n)
    return nums.reshape(n, 3)


def _read_faces(path: str):
    """faceList `n(a b c ...)` entries, or faceCompactList (offsets list + flat label list)"""
    txt = _read(path)
    body = _body(txt)
    if "faceCompactList" in txt:
        n, s = _list_start(body)
        e = body.index(")", s)
        offs = np.array(body[s:e].split(), dtype=np.int64)
        m, s2 = _list_start(body[e + 1:])
        flat = np.array(body[e + 1 + s2:body.index(")", e + 1 + s2)].split(), dtype=np.int64)
        return [flat[offs[i]:offs[i + 1]] for i in range(n - 1)]
    n, s = _list_start(body)
    faces = [np.array(m.group(2).split(), dtype=np.int64) for m in re.finditer(r"(\d+)\s*\(([^()]*)\)", body[s:])]
    assert len(faces) == n, (path, len(faces), n)
    return faces


def _read_boundary(path: str):
    body = _body(_read(path))
    n, s = _list_start(body)
    out = []
    for m in re.finditer(r"(\w+)\s*\{([^{}]*)\}", body[s:]):
        d = dict(re.findall(r"(\w+)\s+([^;]+);", m.group(2)))
        out.append((m.group(1), d))
    assert len(out) == n, (path, len(out), n)
    return out


def face_centres_areas(points: np.ndarray, faces) -> tuple[np.ndarray, np.ndarray]:
    """primitiveMesh::makeFaceCentresAndAreas"""
    F = len(faces)
    Cf = np.zeros((F, 3))
    Sf = np.zeros((F, 3))
    sizes = np.array([len(f) for f in faces])
    for n in np.unique(sizes):
        idx = np.nonzero(sizes == n)[0]
        P = points[np.stack([faces[i] for i in idx])]          # [m, n, 3]
        if n == 3:
            Cf[idx] = P.sum(axis=1) / 3.0
            Sf[idx] = 0.5 * np.cross(P[:, 1] - P[:, 0], P[:, 2] - P[:, 0])
            continue
        fc = P.sum(axis=1) / n
        sumN = np.zeros((len(idx), 3)); sumA = np.zeros(len(idx)); sumAc = np.zeros((len(idx), 3))
        for pi in range(n):
            a, b = P[:, pi], P[:, (pi + 1) % n]
            c = a + b + fc
            nv = np.cross(b - a, fc - a)
            ar = np.linalg.norm(nv, axis=1)
            sumN += nv; sumA += ar; sumAc += ar[:, None] * c
        Cf[idx] = (1.0 / 3.0) * sumAc / np.maximum(sumA, 1e-300)[:, None]
        Sf[idx] = 0.5 * sumN
    return Cf, Sf


def cell_centres_volumes(n_cells, owner, neighbour, Cf, Sf):
    """primitiveMesh::makeCellCentresAndVols (owner covers every face, neighbour the internal ones)"""
    nf = np.bincount(owner, minlength=n_cells) + np.bincount(neighbour, minlength=n_cells)
    cEst = np.zeros((n_cells, 3))
    for k in range(3):
        cEst[:, k] = (np.bincount(owner, Cf[:, k], n_cells) + np.bincount(neighbour, Cf[:neighbour.size, k], n_cells)) / nf
    Fi = neighbour.size
    pyr_o = np.einsum("ij,ij->i", Sf, Cf - cEst[owner])
    pyr_n = np.einsum("ij,ij->i", Sf[:Fi], cEst[neighbour] - Cf[:Fi])
    pc_o = 0.75 * Cf + 0.25 * cEst[owner]
    pc_n = 0.75 * Cf[:Fi] + 0.25 * cEst[neighbour]
    vol = np.bincount(owner, pyr_o, n_cells) + np.bincount(neighbour, pyr_n, n_cells)
    cc = np.zeros((n_cells, 3))
    for k in range(3):
        cc[:, k] = np.bincount(owner, pyr_o * pc_o[:, k], n_cells) + np.bincount(neighbour, pyr_n * pc_n[:, k], n_cells)
    cc /= vol[:, None]
    return cc, vol / 3.0


def read_polymesh(directory: str) -> Mesh:
    """constant/polyMesh (points, faces, owner, neighbour, boundary) -> Mesh"""
    pts = _read_points(os.path.join(directory, "points"))
    faces = _read_faces(os.path.join(directory, "faces"))
    owner = _read_labels(os.path.join(directory, "owner"))
    neighbour = _read_labels(os.path.join(directory, "neighbour"))
    bnd = _read_boundary(os.path.join(directory, "boundary"))
    C = int(max(owner.max(), neighbour.max() if neighbour.size else 0)) + 1
    Fi = neighbour.size
    if Fi and not np.all(np.diff(owner[:Fi].astype(np.int64) * C + neighbour) > 0):
        raise ValueError("polyMesh internal faces are not in upper-triangular order")
    Cf, Sf = face_centres_areas(pts, faces)
    cc, vol = cell_centres_volumes(C, owner, neighbour, Cf, Sf)
    o, n = owner[:Fi], neighbour
    sfi = Sf[:Fi]
    d_o = np.abs(np.einsum("ij,ij->i", sfi, Cf[:Fi] - cc[o]))
    d_n = np.abs(np.einsum("ij,ij->i", sfi, cc[n] - Cf[:Fi]))
    w = d_n / (d_o + d_n)
    mdist = cc[n] - cc[o]
    dcoef = 1.0 / np.linalg.norm(mdist, axis=1)
    magsf = np.linalg.norm(sfi, axis=1)

    patches = []
    names = [b[0] for b in bnd]
    geo = []
    for name, d in bnd:
        nF, s0 = int(d["nFaces"]), int(d["startFace"])
        sl = slice(s0, s0 + nF)
        fc = owner[sl]
        sf = Sf[sl]
        mag = np.linalg.norm(sf, axis=1)
        nfv = sf / np.maximum(mag, 1e-300)[:, None]
        delta = np.einsum("ij,ij->i", nfv, Cf[sl] - cc[fc])[:, None] * nfv   # patch-normal delta (fvPatch::delta)
        geo.append((fc, sf, mag, nfv, delta, Cf[sl] - cc[fc]))
    for pi, (name, d) in enumerate(bnd):
        t = d["type"].strip()
        if t not in _KIND:
            raise ValueError(f"polyMesh patch {name}: type {t} not supported (serial meshes only)")
        kind = _KIND[t]
        fc, sf, mag, nfv, delta, dfull = geo[pi]
        if kind == "empty":
            patches.append(Patch(name, "empty", fc[:0].astype(np.int32), sf[:0], mag[:0], np.ones(0), np.ones(0)))
            continue
        if kind == "cyclic":
            q = names.index(d["neighbourPatch"].strip())
            di = np.einsum("ij,ij->i", nfv, delta)
            dni = np.einsum("ij,ij->i", geo[q][3], geo[q][4])
            wgt = dni / (di + dni)
            # cyclicFvPatch::delta: the full own-side (Cf - C) minus the partner's (translational cyclic)
            dc = 1.0 / np.linalg.norm(dfull - geo[q][5], axis=1)
            p = Patch(name, "cyclic", fc.astype(np.int32), sf, mag, wgt, dc, delta=dfull - geo[q][5])
            p.neighbour_patch = q
        else:
            p = Patch(name, "wall", fc.astype(np.int32), sf, mag, np.ones(fc.size), 1.0 / np.linalg.norm(delta, axis=1),
                      delta=delta)
        patches.append(p)
    return Mesh(n_cells=C, owner=owner[:Fi].astype(np.int32), neighbour=neighbour.astype(np.int32), sf=sfi,
                mag_sf=magsf, weight=w, delta_coeffs=dcoef, volume=vol, cell_centres=cc, mesh_distance=mdist,
                patches=patches, global_offset=0, n_total_cells=C)


# ------------------------------------------------------------------ writer (single hex block)
def _hdr(cls: str, obj: str) -> str:
    return ("FoamFile\n{\n    version     2.0;\n    format      ascii;\n    class       %s;\n"
            "    location    \"constant/polyMesh\";\n    object      %s;\n}\n\n" % (cls, obj))


def hex_polymesh(nx, ny, nz, lengths=(6.283185307179586e-3,) * 3, periodic=(True, True, True),
                 gradings=(1.0, 1.0, 1.0), wall_kinds=None):
    """points, faces, owner, neighbour, boundary [(name, type, nFaces, startFace, neighbourPatch)] of the
    hex box `mesh.hex_box` builds (same cell numbering, same internal-face and patch order)."""
    X = _axis_nodes(nx, lengths[0], gradings[0])
    Y = _axis_nodes(ny, lengths[1], gradings[1])
    Z = _axis_nodes(nz, lengths[2], gradings[2])
    P = np.stack(np.meshgrid(X, Y, Z, indexing="ij"), axis=-1).transpose(2, 1, 0, 3).reshape(-1, 3)
    nid = lambda i, j, k: i + (nx + 1) * (j + (ny + 1) * k)
    cid = lambda i, j, k: i + nx * (j + ny * k)

    def quad(d, i, j, k):   # face at the + side of cell (i, j, k) along axis d, normal +d
        if d == 0: return [nid(i + 1, j, k), nid(i + 1, j + 1, k), nid(i + 1, j + 1, k + 1), nid(i + 1, j, k + 1)]
        if d == 1: return [nid(i, j + 1, k), nid(i, j + 1, k + 1), nid(i + 1, j + 1, k + 1), nid(i + 1, j + 1, k)]
        return [nid(i, j, k + 1), nid(i + 1, j, k + 1), nid(i + 1, j + 1, k + 1), nid(i, j + 1, k + 1)]

    faces, own, nei = [], [], []
    for k in range(nz):
        for j in range(ny):
            for i in range(nx):
                c = cid(i, j, k)
                ent = []
                if i < nx - 1: ent.append((cid(i + 1, j, k), quad(0, i, j, k)))
                if j < ny - 1: ent.append((cid(i, j + 1, k), quad(1, i, j, k)))
                if k < nz - 1: ent.append((cid(i, j, k + 1), quad(2, i, j, k)))
                for nb, f in sorted(ent):
                    faces.append(f); own.append(c); nei.append(nb)
    sides = [("front", 2, +1), ("back", 2, -1), ("left", 0, -1), ("right", 0, +1), ("top", 1, +1), ("down", 1, -1)]
    opp = {"front": "back", "back": "front", "left": "right", "right": "left", "top": "down", "down": "top"}
    wall_kinds = wall_kinds or {}
    n = (nx, ny, nz)
    boundary = []
    for name, axis, side in sides:
        kind = "cyclic" if periodic[axis] else wall_kinds.get(name, "wall")
        ta = [a for a in range(3) if a != axis]
        start = len(faces)
        cnt = 0
        if kind != "empty":
            for t1 in range(n[ta[1]]):
                for t0 in range(n[ta[0]]):
                    ijk = [0, 0, 0]
                    ijk[ta[0]], ijk[ta[1]] = t0, t1
                    ijk[axis] = n[axis] - 1 if side > 0 else 0
                    i, j, k = ijk
                    if side > 0:
                        f = quad(axis, i, j, k)
                    else:
                        m = list(ijk); m[axis] -= 1
                        f = quad(axis, *m)[::-1]
                    faces.append(f); own.append(cid(i, j, k)); cnt += 1
        else:
            # empty patches keep their faces in OpenFOAM; the host arrays drop them (n = 0 slots)
            for t1 in range(n[ta[1]]):
                for t0 in range(n[ta[0]]):
                    ijk = [0, 0, 0]
                    ijk[ta[0]], ijk[ta[1]] = t0, t1
                    ijk[axis] = n[axis] - 1 if side > 0 else 0
                    i, j, k = ijk
                    if side > 0:
                        f = quad(axis, i, j, k)
                    else:
                        m = list(ijk); m[axis] -= 1
                        f = quad(axis, *m)[::-1]
                    faces.append(f); own.append(cid(i, j, k)); cnt += 1
        ftype = {"cyclic": "cyclic", "empty": "empty"}.get(kind, "patch" if kind == "wall" else kind)
        boundary.append((name, ftype, cnt, start, opp[name] if kind == "cyclic" else None))
    return P, faces, np.array(own, np.int32), np.array(nei, np.int32), boundary


def write_polymesh(directory: str, points, faces, owner, neighbour, boundary):
    os.makedirs(directory, exist_ok=True)
    with open(os.path.join(directory, "points"), "w") as f:
        f.write(_hdr("vectorField", "points") + f"{len(points)}\n(\n")
        f.writelines("(%.17g %.17g %.17g)\n" % tuple(p) for p in points)
        f.write(")\n")
    with open(os.path.join(directory, "faces"), "w") as f:
        f.write(_hdr("faceList", "faces") + f"{len(faces)}\n(\n")
        f.writelines("%d(%s)\n" % (len(q), " ".join(str(int(v)) for v in q)) for q in faces)
        f.write(")\n")
    for name, arr in (("owner", owner), ("neighbour", neighbour)):
        with open(os.path.join(directory, name), "w") as f:
            f.write(_hdr("labelList", name) + f"{len(arr)}\n(\n")
            f.writelines("%d\n" % v for v in arr)
            f.write(")\n")
    with open(os.path.join(directory, "boundary"), "w") as f:
        f.write(_hdr("polyBoundaryMesh", "boundary") + f"{len(boundary)}\n(\n")
        for name, t, nF, s0, nbr in boundary:
            f.write(f"    {name}\n    {{\n        type            {t};\n        nFaces          {nF};\n"
                    f"        startFace       {s0};\n")
            if nbr:
                f.write(f"        neighbourPatch  {nbr};\n")
            f.write("    }\n")
        f.write(")\n")
