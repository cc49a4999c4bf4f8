"""Generate deepflame-dev_amd/dfmi/data/mm_collision_tables.json: Omega(2,2)* and A* of the Stockmayer
potential on Cantera's MMCollisionInt grid (37 T* rows x 8 delta* columns), see dfmi/collision.py.

  python scripts/gen_collision_tables.py [--q cross_sections.txt]

Steps: build deepflame-dev_amd/tools/collision_q.c (gcc -O2 -fopenmp), compute Q(1)*(E), Q(2)*(E) for the
fixed-orientation potentials d = -2.5 .. 2.5 (41 values) on 320 energies 3e-4 .. 1e4 (about 15 min on 8
cores), form Omega(1,1)*, Omega(2,2)* per d and T*, average over dipole orientations for each tabulated
delta*, A* = <Omega22> / <Omega11>.

delta* = 0 column above T* = 20: Cantera's table carries the Lennard-Jones values of Hirschfelder, Curtiss
& Bird (Molecular Theory of Gases and Liquids, 1954, Table I-M), whose Omega(2,2)* for T* >= 25 lie
0.03-0.6 % above the exact classical integrals computed here (older quadrature); the reference's table
(thermo_ES80_H2-7-16.txt) was fitted with them (its H2 viscosity up to T* = 92 reproduces them to 1e-4 and
not the exact values). Those seven published Omega(2,2)* values are used as printed; Omega(1,1)* stays the
computed one there (A* = published Omega22 / computed Omega11).
"""
import argparse
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deepflame-dev_amd"))
from dfmi import collision as C    # noqa: E402

# Hirschfelder, Curtiss & Bird (1954) Table I-M, Omega(2,2)* of the 12-6 potential (as carried by Cantera's
# MMCollisionInt omega22_table, delta* = 0 column)
HCB_OMEGA22_HIGH_T = {25.0: 0.7198, 30.0: 0.7010, 35.0: 0.6854, 40.0: 0.6723, 50.0: 0.6510, 75.0: 0.6140,
                      100.0: 0.5887}

D_MIN, D_MAX, N_D = -2.5, 2.5, 41
E_MIN, E_MAX, N_E = 3e-4, 1e4, 320


def cross_sections(path=None):
    if path and os.path.exists(path):
        return np.loadtxt(path)
    src = os.path.join(ROOT, "deepflame-dev_amd", "tools", "collision_q.c")
    exe = os.path.join(ROOT, "deepflame-dev_amd", "tools", "collision_q")
    subprocess.run(["gcc", "-O2", "-fopenmp", "-o", exe, src, "-lm"], check=True)
    out = subprocess.run([exe, str(D_MIN), str(D_MAX), str(N_D), str(E_MIN), str(E_MAX), str(N_E)], check=True,
                         capture_output=True, text=True).stdout
    a = np.loadtxt(out.splitlines())
    if path:
        np.savetxt(path, a)
    return a


def tables(a):
    d_grid = np.unique(np.round(a[:, 0], 10))
    o11 = np.empty((len(d_grid), len(C.TSTAR22)))
    o22 = np.empty_like(o11)
    for i, d in enumerate(d_grid):
        r = a[np.abs(a[:, 0] - d) < 1e-9]
        o11[i] = C.omega_from_cross_sections(r[:, 1], r[:, 2], C.TSTAR22, 1)
        o22[i] = C.omega_from_cross_sections(r[:, 1], r[:, 3], C.TSTAR22, 2)
    om22 = np.empty((37, 8))
    ast = np.empty((37, 8))
    for j, ds in enumerate(C.DELTA):
        a11 = C.orientation_average(d_grid, o11, ds)
        a22 = C.orientation_average(d_grid, o22, ds)
        om22[:, j] = a22
        ast[:, j] = a22 / a11
    exact22 = om22[:, 0].copy()
    for i, t in enumerate(C.TSTAR22):
        if t in HCB_OMEGA22_HIGH_T:   # published Omega22; Omega11 (= Omega22 / A*) stays the computed one
            om22[i, 0] = HCB_OMEGA22_HIGH_T[t]
            ast[i, 0] = om22[i, 0] / (exact22[i] / ast[i, 0])
    return om22, ast, exact22


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--q", default=None, help="cross-section file (read if present, else computed and saved)")
    ap.add_argument("--out", default=C.TABLE_PATH)
    args = ap.parse_args()
    a = cross_sections(args.q)
    om22, ast, exact22 = tables(a)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump({"tstar": C.TSTAR22.tolist(), "delta": C.DELTA.tolist(),
                   "omega22": np.round(om22, 6).tolist(), "astar": np.round(ast, 6).tolist(),
                   "omega22_exact_delta0": np.round(exact22, 6).tolist(),
                   "source": "scripts/gen_collision_tables.py (deepflame-dev_amd/tools/collision_q.c cross sections, "
                             f"d in [{D_MIN}, {D_MAX}] x {N_D}, E in [{E_MIN}, {E_MAX}] x {N_E}; delta*=0 "
                             "Omega22 for T* >= 25 from Hirschfelder-Curtiss-Bird Table I-M)"}, f, indent=0)
    print("wrote", args.out)


if __name__ == "__main__":
    main()
