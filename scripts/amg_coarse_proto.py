#!/usr/bin/env python3
# Round 6, VERDICT r5 item 3: the coarse chain (levels >= 1, ~56 us of latency per V-cycle at 2M cells) against a
# V-cycle that stops one level earlier with more coarsest sweeps. Same operator and V-cycle as amg_sa_proto.py;
# coarsening stops when the next level would be <= `stop`^3 cells; the coarsest level gets `sweeps` Jacobi sweeps.
# python scripts/amg_coarse_proto.py <n> <shift>  (results: profiles/r06_amg_coarse_proto.txt)
import numpy as np, scipy.sparse as sp, sys
n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
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
g = np.exp(0.5 * np.sin(2 * np.pi * np.arange(n**3) / n**3 * 7))
G = sp.diags(np.sqrt(g))
A0 = (G @ lap(n) @ G + shift * sp.diags(g)).tocsr()
OMEGA, SC = 0.9, 1.35
def hierarchy(stop):
    levels = []; A = A0; nn = n
    while nn > stop:
        P = agg(nn); levels.append((A, P)); A = (P.T @ A @ P).tocsr(); nn //= 2
    levels.append((A, None))
    return levels
def jacobi(A, b, x, sweeps):
    D = A.diagonal()
    for _ in range(sweeps):
        x = x + OMEGA * (b - A @ x) / D
    return x
def vcycle(levels, l, b, sweeps):
    A, P = levels[l]
    if P is None:
        return jacobi(A, b, np.zeros_like(b), sweeps)
    x = jacobi(A, b, np.zeros_like(b), 1)
    xc = vcycle(levels, l + 1, P.T @ (b - A @ x), sweeps)
    return jacobi(A, b, x + SC * (P @ xc), 1)
def pcg(levels, sweeps, tol=1e-5):
    b = rng.standard_normal(n**3)
    x = np.zeros_like(b); r = b - A0 @ x; r0 = np.linalg.norm(r)
    z = vcycle(levels, 0, r, sweeps); p = z.copy(); rz = r @ z
    for it in range(1, 300):
        q = A0 @ p; a = rz / (p @ q); x += a * p; r -= a * q
        if np.linalg.norm(r) <= tol * r0: return it
        z = vcycle(levels, 0, r, sweeps); rzn = r @ z; p = z + rzn / rz * p; rz = rzn
    return -1
for stop in (8, 16):
    lv = hierarchy(stop)
    for sweeps in ((8,) if stop == 8 else (8, 16, 32, 64)):
        print(n, shift, "levels", len(lv), "coarsest", lv[-1][0].shape[0], "sweeps", sweeps, "iterations",
              pcg(lv, sweeps), flush=True)
