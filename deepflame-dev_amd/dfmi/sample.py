"""Line sampling with OpenFOAM-7's cellPoint interpolation on blockMesh hex boxes.

The reference's regression values are sampled this way: test/dfLowMachFoam/twoD_reactingTGV/H2/
cvodeSolver/system/sample (type sets, lineUniform, interpolationScheme cellPoint, setFormat raw) writes
postProcessing/sample/<t>/data_T.xy, and test/corrtest.cpp:20-24,131-156 reads single values out of it.

Restated from OpenFOAM-7:
  * volPointInterpolation: point value = sum over the point's cells of w_c psi_c / sum w_c with
    w_c = 1/|p - C_c|; points on empty and coupled patches are not "patch points" (calcBoundaryAddressing),
    so they take these internal weights, summed across cyclic partners (syncPointList);
  * interpolationCellPoint / cellPointWeight::findTetrahedron: the cell is cut into tets (cell centre,
    face base point, two consecutive face points) with the face's first point as base
    (polyMeshTetDecomposition::findBasePoint returns point 0 of every well-shaped hex face); the value is
    the barycentric combination of the cell value and the three point values of the tet holding the
    sample point;
  * blockMesh numbering: points i fastest then j then k, cells likewise, every face's point list the hex
    model face of its owner (boundary faces the cell's own face; polyMeshFromShapeMesh). The hex model
    faces are (0 4 7 3) (1 2 6 5) (0 1 5 4) (3 7 6 2) (0 3 2 1) (4 5 6 7); the base point of a face shared
    by two cells is the same point from either side.
"""
from __future__ import annotations

import numpy as np

HEX_FACES = ((0, 4, 7, 3), (1, 2, 6, 5), (0, 1, 5, 4), (3, 7, 6, 2), (0, 3, 2, 1), (4, 5, 6, 7))


class CellPointSampler:
    """cellPoint interpolation of cell fields of a single-block blockMesh box (hex_box)."""

    def __init__(self, m, nodes, periodic):
        """nodes: the three node-coordinate arrays (x, y, z) of the block; periodic: per axis"""
        self.m = m
        self.X = [np.asarray(a, dtype=np.float64) for a in nodes]
        self.n = [len(a) - 1 for a in self.X]
        self.periodic = periodic
        nx, ny, nz = self.n
        assert nx * ny * nz == m.n_cells
        ii, jj, kk = m.local_index
        self.cid = np.zeros((nx, ny, nz), dtype=np.int64)
        self.cid[ii, jj, kk] = np.arange(m.n_cells)
        self.cc = m.cell_centres

    def _point_cells(self, i, j, k):
        """cells around node (i, j, k) and the centres as seen from the node (periodic images)"""
        out = []
        for di in (-1, 0):
            for dj in (-1, 0):
                for dk in (-1, 0):
                    idx = [i + di, j + dj, k + dk]
                    shift = np.zeros(3)
                    ok = True
                    for a in range(3):
                        if idx[a] < 0 or idx[a] >= self.n[a]:
                            if not self.periodic[a]:
                                ok = False
                                break
                            L = self.X[a][-1] - self.X[a][0]
                            shift[a] = -L if idx[a] < 0 else L
                            idx[a] %= self.n[a]
                    if ok:
                        c = self.cid[idx[0], idx[1], idx[2]]
                        out.append((c, self.cc[c] + shift))
        return out

    def point_value(self, psi, i, j, k):
        p = np.array([self.X[0][i], self.X[1][j], self.X[2][k]])
        num = 0.0
        den = 0.0
        for c, cen in self._point_cells(i, j, k):
            w = 1.0 / np.linalg.norm(p - cen)
            num += w * psi[c]
            den += w
        return num / den

    def interpolate(self, psi, pos):
        """value of cell field psi [C] at position pos [3]"""
        pos = np.asarray(pos, dtype=np.float64)
        ijk = []
        for a in range(3):
            t = int(np.searchsorted(self.X[a], pos[a], side="right") - 1)
            ijk.append(min(max(t, 0), self.n[a] - 1))
        i, j, k = ijk
        c = self.cid[i, j, k]
        verts = [(i, j, k), (i + 1, j, k), (i + 1, j + 1, k), (i, j + 1, k),
                 (i, j, k + 1), (i + 1, j, k + 1), (i + 1, j + 1, k + 1), (i, j + 1, k + 1)]
        P = np.array([[self.X[0][a], self.X[1][b], self.X[2][d]] for a, b, d in verts])
        cen = self.cc[c]
        best = None
        tol = 1e-10
        for f in HEX_FACES:
            for t in range(1, len(f) - 1):
                tri = (f[0], f[t], f[t + 1])
                A = np.stack([P[tri[0]] - cen, P[tri[1]] - cen, P[tri[2]] - cen], axis=1)
                lam = np.linalg.solve(A, pos - cen)
                w = np.array([1.0 - lam.sum(), lam[0], lam[1], lam[2]])
                if np.all(w > -tol):
                    val = w[0] * psi[c] + sum(w[q + 1] * self.point_value(psi, *verts[tri[q]]) for q in range(3))
                    return val
                score = w.min()
                if best is None or score > best[0]:
                    best = (score, tri, w)
        # not inside any tet within tolerance (numerically on an edge): the least-outside one
        _, tri, w = best
        return w[0] * psi[c] + sum(w[q + 1] * self.point_value(psi, *verts[tri[q]]) for q in range(3))

    def line_uniform(self, psi, start, end, n_points):
        """OpenFOAM lineUniform set: n_points equally spaced from start to end (inclusive)"""
        s = np.asarray(start, dtype=np.float64)
        e = np.asarray(end, dtype=np.float64)
        pts = [s + (e - s) * q / (n_points - 1) for q in range(n_points)]
        return np.array(pts), np.array([self.interpolate(psi, p) for p in pts])


def raw_token_value(points_axis, values, k):
    """the k-th whitespace token (1-based) of the raw-format set file "axis value" per line, as
    test/corrtest.cpp readTGV counts them (corrtest.cpp:131-156)"""
    toks = np.stack([points_axis, values], axis=1).ravel()
    return float(toks[k - 1])
