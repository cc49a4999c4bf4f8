#!/usr/bin/env python3
# Round 6, VERDICT r5 item 3: would a smoothed-aggregation prolongator between levels 0 and 1 pay?
# python scripts/amg_sa_proto.py <n> <shift>  (results: profiles/r06_amg_sa_proto.txt)
# The p equation's shape (shifted 7-point Laplacian, shift ~ psi/dt vs the laplacian: 1e-2 .. 1e-3), PCG to 1e-5 with
# the production V-cycle (2x2x2 pairwise aggregates, one weighted-Jacobi sweep w = 0.9 before and after, coarse
# correction x 1.35, 8 Jacobi sweeps on the coarsest) against the same V-cycle whose level-0 -> 1 prolongator is
# smoothed: P = (I - w_p D^-1 A) P0, w_p = 4 / (3 lambda_max(D^-1 A)), A1 = P^T A P (27-point), no over-correction
# on that level. Reports PCG iterations and the level-1 operator's width (the cost side of the trade).
import numpy as np, scipy.sparse as sp, sys
n = int(sys.argv[1]) if len(sys.argv) > 1 else 32
shift = float(sys.argv[2]) if len(sys.argv) > 2 else 0.01
def lap(n):
    I = sp.identity(n); e = np.ones(n)
    T = sp.diags([-e[:-1], 2*e, -e[:-1]], [-1, 0, 1]).tolil()
    T[0, n-1] = -1; T[n-1, 0] = -1
    T = T.tocsr()
    return (sp.kron(sp.kron(T, I), I) + sp.kron(sp.kron(I, T), I) + sp.kron(sp.kron(I, I), T)).tocsr()
def agg(n):
    i = np.arange(n)
    ii, jj, kk = np.meshgrid(i, i, i, indexing='ij')
    m = n // 2
    a = (ii//2)*m*m + (jj//2)*m + kk//2
    return sp.csr_matrix((np.ones(n**3), (a.ravel(), np.arange(n**3))), shape=(m**3, n**3)).T.tocsr()
rng = np.random.default_rng(0)
# smoothly varying coefficients, like rho rAU across a flame: a symmetric diagonal scaling of the laplacian
g = np.exp(0.5 * np.sin(2 * np.pi * np.arange(n**3) / n**3 * 7))
G = sp.diags(np.sqrt(g))
A0 = (G @ lap(n) @ G + shift * sp.diags(g)).tocsr()
def lmax(A):
    D = A.diagonal(); v = rng.random(A.shape[0])
    for _ in range(40): v = (A @ v) / D; v /= np.linalg.norm(v)
    return float(v @ ((A @ v) / D))
def hierarchy(sa):
    levels = []; A = A0; nn = n; l = 0
    while nn > 8:
        P = agg(nn)
        sc = 1.35
        if sa and l == 0:
            D = A.diagonal(); wp = 4.0 / (3.0 * lmax(A))
            P = (P - wp * sp.diags(1.0 / D) @ (A @ P)).tocsr()
            sc = 1.0
        Ac = (P.T @ A @ P).tocsr()
        levels.append((A, P, sc)); A = Ac; nn //= 2; l += 1
    levels.append((A, None, 1.0))
    return levels
OMEGA = 0.9
def jacobi(A, b, x, sweeps):
    D = A.diagonal()
    for _ in range(sweeps):
        x = x + OMEGA * (b - A @ x) / D
    return x
def vcycle(levels, l, b):
    A, P, sc = levels[l]
    if P is None:
        return jacobi(A, b, np.zeros_like(b), 8)
    x = jacobi(A, b, np.zeros_like(b), 1)
    xc = vcycle(levels, l + 1, P.T @ (b - A @ x))
    return jacobi(A, b, x + sc * (P @ xc), 1)
def pcg(levels, tol=1e-5):
    b = rng.standard_normal(n**3)
    x = np.zeros_like(b); r = b - A0 @ x; r0 = np.linalg.norm(r)
    z = vcycle(levels, 0, r); p = z.copy(); rz = r @ z
    for it in range(1, 300):
        q = A0 @ p; a = rz / (p @ q); x += a * p; r -= a * q
        if np.linalg.norm(r) <= tol * r0: return it
        z = vcycle(levels, 0, r); rzn = r @ z; p = z + rzn / rz * p; rz = rzn
    return -1
for sa in (False, True):
    lv = hierarchy(sa)
    w1 = np.diff(lv[1][0].indptr).max() - 1
    print(n, shift, "smoothed-l0" if sa else "plain", "iterations", pcg(lv), "level-1 width", w1, flush=True)
