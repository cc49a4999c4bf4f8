"""Structured hex-box mesh in OpenFOAM polyMesh/lduAddressing conventions.

This is the host-side input builder that stands in for what OpenFOAM hands the
GPU path in ``createGPUBase`` (reference ``applications/solvers/dfLowMachFoam/
createGPUSolver.H:103-351``): owner/neighbour in upper-triangular face order,
face area vectors (AoS, as ``mesh.Sf()``), magSf, linear-interpolation weights,
deltaCoeffs, cell volumes, and the flattened boundary arrays in patch order
where a processor/processorCyclic patch takes ``2*n`` slots
``[neighbour values | patch-internal values]`` (``createGPUSolver.H:265-304``).

Geometry follows OpenFOAM ``surfaceInterpolation``:
  * internal weight  w = (Sf.(Cn-Cf)) / (Sf.(Cf-Co) + Sf.(Cn-Cf))
  * deltaCoeffs      1/|Cn - Co|
  * non-coupled patch: w = 1, deltaCoeffs = 1/|Cf - Co|
  * cyclic/processor patch: w = dn/(d + dn), deltaCoeffs = 1/(d + dn)
    (``cyclicFvPatch::makeWeights`` / ``coupledFvPatch::delta``).

The blockMesh pattern is that of the reference GPU example
``examples/dfLowMachFoam/notorch/threeD_reactingTGV/H2/cvodeIntegrator/system/
blockMeshDict:34-90`` (single hex block, 6 patches front/back/left/right/top/down).
"""
from __future__ import annotations

from dataclasses import dataclass, field
import numpy as np

# reference patch-type codes (dfMatrixDataBase.H:81-93)
ZERO_GRADIENT = 0
FIXED_VALUE = 1
COUPLED = 2
EMPTY = 3
GRADIENT_ENERGY = 4
CALCULATED = 5
CYCLIC = 6
PROCESSOR = 7
EXTRAPOLATED = 8
FIXED_ENERGY = 9
PROCESSOR_CYCLIC = 10
WAVE_TRANSMISSIVE = 11   # mixed conditions beyond the reference GPU enum (include/dfmi.h)
INLET_OUTLET = 12

BC_NAMES = {
    "zeroGradient": ZERO_GRADIENT, "fixedValue": FIXED_VALUE, "coupled": COUPLED,
    "empty": EMPTY, "gradientEnergy": GRADIENT_ENERGY, "calculated": CALCULATED,
    "cyclic": CYCLIC, "processor": PROCESSOR, "extrapolated": EXTRAPOLATED,
    "fixedEnergy": FIXED_ENERGY, "processorCyclic": PROCESSOR_CYCLIC,
    "waveTransmissive": WAVE_TRANSMISSIVE, "inletOutlet": INLET_OUTLET,
}


@dataclass
class Patch:
    name: str
    kind: str                 # "wall" | "cyclic" | "processor" | "processorCyclic" | "empty"
    face_cells: np.ndarray    # int32 [n]
    sf: np.ndarray            # [n,3] outward area vectors
    mag_sf: np.ndarray
    weight: np.ndarray
    delta_coeffs: np.ndarray
    neighbour_patch: int = -1     # cyclic partner patch index
    peer_rank: int = -1           # processor neighbour rank
    peer_patch: int = -1          # index of the matching patch on peer_rank
    nbr_cells_global: np.ndarray | None = None  # procCols (global ids of cells across the patch)
    # [n,3] patch delta vectors (fvPatch::delta; coupled: (Cf - C) - (Cf' - C'), cyclicFvPatch::delta /
    # processorFvPatch::delta), the d the limited schemes' limiter reads across a coupled face
    # (LimitedScheme::calcLimiter); None: the patch-normal n/deltaCoeffs of an orthogonal patch
    delta: np.ndarray | None = None

    @property
    def size(self) -> int:
        return int(self.face_cells.shape[0])

    @property
    def slots(self) -> int:
        return 2 * self.size if self.kind in ("processor", "processorCyclic") else self.size


@dataclass
class Mesh:
    n_cells: int
    owner: np.ndarray          # int32 [F]
    neighbour: np.ndarray      # int32 [F]
    sf: np.ndarray             # [F,3]
    mag_sf: np.ndarray
    weight: np.ndarray
    delta_coeffs: np.ndarray
    volume: np.ndarray         # [C]
    cell_centres: np.ndarray   # [C,3]
    mesh_distance: np.ndarray  # [F,3] C[nei]-C[own]
    patches: list = field(default_factory=list)
    global_offset: int = 0     # first global cell id of this rank
    n_total_cells: int = 0

    @property
    def n_faces(self) -> int:
        return int(self.owner.shape[0])

    @property
    def n_patches(self) -> int:
        return len(self.patches)

    @property
    def n_boundary_slots(self) -> int:
        return int(sum(p.slots for p in self.patches))

    @property
    def n_coupled_slots(self) -> int:
        """primary slots of coupled patches (cyclic / processor): one off-diagonal matrix entry each"""
        return int(sum(p.size for p in self.patches if p.kind in ("cyclic", "processor", "processorCyclic")))

    @property
    def patch_sizes(self) -> np.ndarray:
        return np.array([p.size for p in self.patches], dtype=np.int32)

    def cyclic_neighbour(self) -> np.ndarray:
        return np.array([p.neighbour_patch for p in self.patches], dtype=np.int32)

    def neighb_proc_no(self) -> np.ndarray:
        return np.array([p.peer_rank for p in self.patches], dtype=np.int32)

    def boundary_arrays(self):
        """Flattened boundary arrays exactly as createGPUBase builds them."""
        sf, mag, dc, w, fc = [], [], [], [], []
        for p in self.patches:
            reps = 2 if p.kind in ("processor", "processorCyclic") else 1
            for _ in range(reps):
                sf.append(p.sf); mag.append(p.mag_sf); dc.append(p.delta_coeffs)
                w.append(p.weight); fc.append(p.face_cells)
        if not sf:
            z = np.zeros(0)
            return np.zeros((0, 3)), z, z, z, np.zeros(0, np.int32)
        return (np.concatenate(sf), np.concatenate(mag), np.concatenate(dc),
                np.concatenate(w), np.concatenate(fc).astype(np.int32))

    def boundary_delta(self) -> np.ndarray:
        """[B,3] patch delta vectors per boundary slot (processor patches: both halves)"""
        out = []
        for p in self.patches:
            reps = 2 if p.kind in ("processor", "processorCyclic") else 1
            if p.delta is not None:
                dv = np.asarray(p.delta, dtype=np.float64).reshape(-1, 3)
            else:
                nf = p.sf / np.maximum(p.mag_sf, 1e-300)[:, None] if p.size else np.zeros((0, 3))
                dv = nf / p.delta_coeffs[:, None] if p.size else np.zeros((0, 3))
            out += [dv] * reps
        return np.concatenate(out) if out else np.zeros((0, 3))

    def proc_rows_cols(self):
        """procRows/procCols for processor interfaces (createGPUSolver.H:205-243)."""
        rows, cols = [], []
        for p in self.patches:
            if p.kind in ("processor", "processorCyclic"):
                rows.append(p.face_cells)
                cols.append(p.nbr_cells_global)
        if not rows:
            return np.zeros(0, np.int32), np.zeros(0, np.int32)
        return np.concatenate(rows).astype(np.int32), np.concatenate(cols).astype(np.int32)

    def patch_types(self, wall_type: int) -> np.ndarray:
        """Per-patch BC code for a field whose physical walls use ``wall_type``."""
        out = []
        for p in self.patches:
            out.append({"cyclic": CYCLIC, "processor": PROCESSOR,
                        "processorCyclic": PROCESSOR_CYCLIC, "empty": EMPTY}.get(p.kind, wall_type))
        return np.array(out, dtype=np.int32)

    def derived_patch_types(self, default: int) -> np.ndarray:
        """patch_type_calculated / patch_type_extrapolated lists (createGPUSolver.H:260-304)."""
        return self.patch_types(default)


def _axis_nodes(n: int, length: float, grading=1.0) -> np.ndarray:
    """Node coordinates of one block edge. `grading` is blockMesh's simpleGrading entry for the
    axis: an expansion ratio (last / first cell size), or a multi-grading list of sections
    (length fraction, cell fraction, expansion ratio), e.g. the 1D flame's
    ((0.55 0.625 1) (0.45 0.375 2)) (test/Tu500K-Phi1/system/blockMeshDict)."""
    if np.ndim(grading) == 0:
        grading = [(1.0, 1.0, float(grading))]
    secs = np.asarray(grading, dtype=np.float64)
    lf = secs[:, 0] / secs[:, 0].sum()
    cf = secs[:, 1] / secs[:, 1].sum()
    counts = np.rint(cf * n).astype(int)
    counts[-1] = n - counts[:-1].sum()
    sizes = []
    for (_, _, ratio), nc, L in zip(secs, counts, lf * length):
        if nc == 0:
            continue
        r = ratio ** (1.0 / (nc - 1)) if nc > 1 else 1.0
        d = np.array([r ** i for i in range(nc)])
        sizes.append(d / d.sum() * L)
    d = np.concatenate(sizes)
    x = np.concatenate([[0.0], np.cumsum(d)])
    x[-1] = length
    return x


def hex_box(nx: int, ny: int, nz: int, lengths=(6.283185307179586e-3,) * 3,
            periodic=(True, True, True), gradings=(1.0, 1.0, 1.0),
            decomp=(1, 1, 1), rank: int = 0, wall_kinds=None) -> Mesh:
    """Hex box (optionally a rank's block of a px*py*pz decomposition).

    Cells are numbered i fastest, then j, then k (blockMesh order). Internal
    faces are emitted per owner cell towards +x, +y, +z neighbours, which is the
    upper-triangular order OpenFOAM requires. Patches follow the reference
    blockMeshDict order: front(z+), back(z-), left(x-), right(x+), top(y+),
    down(y-). On a decomposed box, sides shared with another rank become
    ``processor`` patches (``processorCyclic`` across a periodic wrap) appended
    after the physical patches, one per neighbouring side, as decomposePar does.
    """
    px, py, pz = decomp
    nranks = px * py * pz
    assert 0 <= rank < nranks
    assert nx % px == 0 and ny % py == 0 and nz % pz == 0
    rx, ry, rz = rank % px, (rank // px) % py, rank // (px * py)
    lnx, lny, lnz = nx // px, ny // py, nz // pz
    X = _axis_nodes(nx, lengths[0], gradings[0])
    Y = _axis_nodes(ny, lengths[1], gradings[1])
    Z = _axis_nodes(nz, lengths[2], gradings[2])
    xs, ys, zs = X[rx * lnx:(rx + 1) * lnx + 1], Y[ry * lny:(ry + 1) * lny + 1], Z[rz * lnz:(rz + 1) * lnz + 1]
    glob = [X, Y, Z]
    loc = [xs, ys, zs]
    ln = [lnx, lny, lnz]
    nper = [px, py, pz]
    rpos = [rx, ry, rz]

    def centres(nodes):
        return 0.5 * (nodes[:-1] + nodes[1:])

    cx, cy, cz = centres(xs), centres(ys), centres(zs)
    dx, dy, dz = np.diff(xs), np.diff(ys), np.diff(zs)
    C = lnx * lny * lnz
    I, J, K = np.meshgrid(np.arange(lnx), np.arange(lny), np.arange(lnz), indexing="ij")
    # cell id = i + lnx*(j + lny*k)
    cid = lambda i, j, k: i + lnx * (j + lny * k)
    kk, jj, ii = np.meshgrid(np.arange(lnz), np.arange(lny), np.arange(lnx), indexing="ij")
    ii = ii.ravel(); jj = jj.ravel(); kk = kk.ravel()  # in cell order
    vol = dx[ii] * dy[jj] * dz[kk]
    cc = np.stack([cx[ii], cy[jj], cz[kk]], axis=1)

    # internal faces in upper-triangular order: per cell, +x, +y, +z
    own_l, nei_l, dir_l = [], [], []
    cells = np.arange(C)
    for d in range(3):
        idx = [ii, jj, kk][d]
        m = idx < ln[d] - 1
        stride = [1, lnx, lnx * lny][d]
        own_l.append(cells[m]); nei_l.append(cells[m] + stride); dir_l.append(np.full(m.sum(), d))
    own = np.concatenate(own_l); nei = np.concatenate(nei_l); fdir = np.concatenate(dir_l)
    order = np.lexsort((nei, own))
    own, nei, fdir = own[order], nei[order], fdir[order]
    F = own.shape[0]
    area = [dy[jj] * dz[kk], dx[ii] * dz[kk], dx[ii] * dy[jj]]
    sf = np.zeros((F, 3))
    magsf = np.zeros(F)
    w = np.zeros(F)
    dcoef = np.zeros(F)
    cen = [cx, cy, cz]
    node = [xs, ys, zs]
    for d in range(3):
        m = fdir == d
        o = own[m]
        oi = [ii, jj, kk][d][o]
        a = area[d][o]
        sf[m, d] = a
        magsf[m] = a
        cf = node[d][oi + 1]
        do = cf - cen[d][oi]
        dn = cen[d][oi + 1] - cf
        w[m] = dn / (do + dn)
        dcoef[m] = 1.0 / (cen[d][oi + 1] - cen[d][oi])
    mdist = cc[nei] - cc[own]

    patches: list[Patch] = []
    # side definitions: (name, axis, side(+1 max / -1 min))
    sides = [("front", 2, +1), ("back", 2, -1), ("left", 0, -1), ("right", 0, +1), ("top", 1, +1), ("down", 1, -1)]
    wall_kinds = wall_kinds or {}

    def side_cells(axis, side):
        idx = [ii, jj, kk][axis]
        target = ln[axis] - 1 if side > 0 else 0
        m = idx == target
        c = cells[m]
        # tangential ordering: (other axes) lexicographic so partner faces match
        ta = [a for a in range(3) if a != axis]
        t0 = [ii, jj, kk][ta[0]][m]; t1 = [ii, jj, kk][ta[1]][m]
        o = np.lexsort((t0, t1))
        return c[o]

    def side_geom(axis, side, fc):
        n = fc.shape[0]
        a = area[axis][fc]
        s = np.zeros((n, 3)); s[:, axis] = side * a
        idx = [ii, jj, kk][axis][fc]
        cf = node[axis][idx + 1] if side > 0 else node[axis][idx]
        d_own = np.abs(cf - cen[axis][idx])
        return s, a, d_own

    def rank_of(r3):
        return r3[0] + px * (r3[1] + py * r3[2])

    phys_sides = []
    proc_sides = []
    for si, (name, axis, side) in enumerate(sides):
        at_domain_edge = (rpos[axis] == nper[axis] - 1) if side > 0 else (rpos[axis] == 0)
        if nper[axis] == 1 and periodic[axis]:
            phys_sides.append((si, name, axis, side, "cyclic"))
        elif at_domain_edge and not periodic[axis]:
            phys_sides.append((si, name, axis, side, wall_kinds.get(name, "wall")))
        else:
            # shared with another rank (possibly across the periodic wrap)
            if nper[axis] == 1:
                continue
            nb = list(rpos)
            nb[axis] = (rpos[axis] + side) % nper[axis]
            kind = "processorCyclic" if at_domain_edge else "processor"
            proc_sides.append((si, name, axis, side, kind, rank_of(nb)))

    name_to_idx = {}
    for (si, name, axis, side, kind) in phys_sides:
        fc = side_cells(axis, side)
        s, a, d_own = side_geom(axis, side, fc)
        if kind == "cyclic":
            # partner across the box: same d on the other side
            osi = {"front": "back", "back": "front", "left": "right", "right": "left", "top": "down", "down": "top"}[name]
            ofc = side_cells(axis, -side)
            _, _, d_nbr = side_geom(axis, -side, ofc)
            wgt = d_nbr / (d_own + d_nbr)
            dc = 1.0 / (d_own + d_nbr)
        elif kind == "empty":
            fc = fc[:0]; s = s[:0]; a = a[:0]; d_own = d_own[:0]
            wgt = np.ones(0); dc = np.ones(0)
        else:
            wgt = np.ones(fc.shape[0])
            dc = 1.0 / d_own
        name_to_idx[name] = len(patches)
        dv = np.zeros((fc.shape[0], 3))
        dv[:, axis] = side * (d_own + d_nbr) if kind == "cyclic" else side * d_own
        patches.append(Patch(name, kind, fc.astype(np.int32), s, a, wgt, dc, delta=dv))
    for p in patches:
        if p.kind == "cyclic":
            osi = {"front": "back", "back": "front", "left": "right", "right": "left", "top": "down", "down": "top"}[p.name]
            p.neighbour_patch = name_to_idx[osi]

    for (si, name, axis, side, kind, peer) in proc_sides:
        fc = side_cells(axis, side)
        s, a, d_own = side_geom(axis, side, fc)
        # neighbour cells on the peer: the opposite side layer of its block
        li, lj, lk = ii[fc].copy(), jj[fc].copy(), kk[fc].copy()
        lidx = [li, lj, lk]
        lidx[axis] = np.full_like(lidx[axis], 0 if side > 0 else ln[axis] - 1)
        # OpenFOAM globalIndex numbering: rank-blocked, offset = peer * C
        gids = peer * C + cid(*lidx)
        # neighbour-side distance from the face to the peer cell centre
        gidx = rpos[axis] * ln[axis] + [ii, jj, kk][axis][fc]
        gn = glob[axis]
        gcen = 0.5 * (gn[:-1] + gn[1:])
        nb_g = (gidx + side) % (len(gn) - 1)
        d_nbr = (gcen[nb_g] - gn[nb_g]) if side > 0 else (gn[nb_g + 1] - gcen[nb_g])
        d_nbr = np.abs(d_nbr)
        wgt = d_nbr / (d_own + d_nbr)
        dc = 1.0 / (d_own + d_nbr)
        dv = np.zeros((fc.shape[0], 3))
        dv[:, axis] = side * (d_own + d_nbr)
        p = Patch(f"procBoundary{rank}to{peer}_{name}", kind, fc.astype(np.int32), s, a, wgt, dc,
                  peer_rank=peer, delta=dv)
        p.nbr_cells_global = gids.astype(np.int32)
        p.side = (axis, side)
        patches.append(p)

    m = Mesh(n_cells=C, owner=own.astype(np.int32), neighbour=nei.astype(np.int32), sf=sf, mag_sf=magsf,
             weight=w, delta_coeffs=dcoef, volume=vol, cell_centres=cc, mesh_distance=mdist, patches=patches,
             global_offset=rank * C, n_total_cells=C * nranks)
    m.local_index = (ii, jj, kk)
    m.nodes = (xs, ys, zs)
    m.block = (rx, ry, rz)
    m.block_dims = (lnx, lny, lnz)
    return m


def global_cell_ids(m: Mesh, nx: int, ny: int) -> np.ndarray:
    ii, jj, kk = m.local_index
    lnx, lny, lnz = m.block_dims
    rx, ry, rz = m.block
    return (rx * lnx + ii) + nx * ((ry * lny + jj) + ny * (rz * lnz + kk))
