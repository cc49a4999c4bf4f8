#!/usr/bin/env python3
# Round 5, VERDICT r4 item 4: does a degree-2 Chebyshev level-0 smoother beat weighted Jacobi on iterations x cost?
# python scripts/amg_smoother_proto.py <n> <shift>  (results: profiles/r05_amg_smoother_proto.txt)
# PCG with a plain-aggregation (2x2x2) V-cycle on a shifted 7-point Laplacian (the p equation's shape: laplacian
# + psi/dt diagonal, ratio ~1/100): level-0 smoother = weighted Jacobi (1 or 2 sweeps) vs Chebyshev degree 2/3
import numpy as np, scipy.sparse as sp, scipy.sparse.linalg as spl, sys
n = int(sys.argv[1]) if len(sys.argv) > 1 else 32
shift = float(sys.argv[2]) if len(sys.argv) > 2 else 0.01
def lap(n, periodic=True):
    I = sp.identity(n); e = np.ones(n)
    T = sp.diags([-e[:-1], 2*e, -e[:-1]], [-1, 0, 1]).tolil()
    if periodic: T[0, n-1] = -1; T[n-1, 0] = -1
    T = T.tocsr()
    A = sp.kron(sp.kron(T, I), I) + sp.kron(sp.kron(I, T), I) + sp.kron(sp.kron(I, I), T)
    return A.tocsr()
def agg(n):
    i = np.arange(n)
    ii, jj, kk = np.meshgrid(i, i, i, indexing='ij')
    m = n // 2
    a = (ii//2)*m*m + (jj//2)*m + kk//2
    P = sp.csr_matrix((np.ones(n**3), (a.ravel(), np.arange(n**3))), shape=(m**3, n**3)).T.tocsr()
    return P
rng = np.random.default_rng(0)
# variable coefficients like rhorAUf ~ rho * rAU varying smoothly
A0 = lap(n) + shift * sp.identity(n**3)
levels = []
A = A0; nn = n
while nn > 8:
    P = agg(nn); Ac = (P.T @ A @ P).tocsr()
    levels.append((A, P)); A = Ac; nn //= 2
levels.append((A, None))
OMEGA, SC = 0.9, 1.35
def jacobi(A, b, x, sweeps):
    D = A.diagonal()
    for _ in range(sweeps):
        x = x + OMEGA * (b - A @ x) / D
    return x
def cheb(A, b, x, deg, lmax):
    # Chebyshev smoother on D^-1 A over [lmax/30, lmax] (standard smoothing interval)
    D = A.diagonal(); lmin = lmax / 30.0
    theta = 0.5 * (lmax + lmin); delta = 0.5 * (lmax - lmin)
    sigma = theta / delta; rho = 1.0 / sigma
    r = (b - A @ x) / D
    d = r / theta
    for k in range(deg):
        x = x + d
        if k == deg - 1: break
        r = r - (A @ d) / D
        rho_n = 1.0 / (2 * sigma - rho)
        d = rho_n * rho * d + 2 * rho_n / delta * r
        rho = rho_n
    return x
lmaxs = []
for A, P in levels:
    D = A.diagonal()
    v = rng.random(A.shape[0])
    for _ in range(30): v = (A @ v) / D; v /= np.linalg.norm(v)
    lmaxs.append(float(v @ ((A @ v) / D)) * 1.05)
def vcycle(l, b, smoother):
    A, P = levels[l]
    if P is None:
        x = np.zeros_like(b)
        return jacobi(A, b, x, 8)
    x = smoother(A, b, np.zeros_like(b), l)
    r = b - A @ x
    xc = vcycle(l + 1, P.T @ r, smoother)
    x = x + SC * (P @ xc)
    return smoother(A, b, x, l)
def pcg(smoother, tol=1e-5):
    b = rng.standard_normal(n**3); b -= b.mean() if shift == 0 else 0
    x = np.zeros_like(b); r = b - A0 @ x; r0 = np.linalg.norm(r)
    z = vcycle(0, r, smoother); p = z.copy(); rz = r @ z
    for it in range(1, 200):
        q = A0 @ p; a = rz / (p @ q); x += a * p; r -= a * q
        if np.linalg.norm(r) <= tol * r0: return it
        z = vcycle(0, r, smoother); rzn = r @ z; p = z + rzn / rz * p; rz = rzn
    return -1
sm = {
  "jacobi1": lambda A, b, x, l: jacobi(A, b, x, 1),
  "jacobi2@l0": lambda A, b, x, l: jacobi(A, b, x, 2 if l == 0 else 1),
  "cheb2@l0": lambda A, b, x, l: cheb(A, b, x, 2, lmaxs[l]) if l == 0 else jacobi(A, b, x, 1),
  "cheb3@l0": lambda A, b, x, l: cheb(A, b, x, 3, lmaxs[l]) if l == 0 else jacobi(A, b, x, 1),
  "cheb2@all": lambda A, b, x, l: cheb(A, b, x, 2, lmaxs[l]),
}
for k, f in sm.items():
    print(n, shift, k, pcg(f), flush=True)
