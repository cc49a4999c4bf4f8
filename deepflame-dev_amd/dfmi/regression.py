"""The reference's whole-loop regression cases, run through the C ABI.

2D reacting Taylor-Green vortex (test/dfLowMachFoam/twoD_reactingTGV/H2/cvodeSolver, committed as
tests/golden/tgv2d): 128 x 128 x 1 cells of a 2 pi mm box (system/blockMeshDict), cyclic in x and y, empty
front/back, ES80 7 species (H2/air), dt = 1e-6 s, 500 steps (system/controlDict), nOuter 1 / nCorr 2
(system/fvSolution:83-84), divSchemes Yi_h limitedLinear01 1 / K limitedLinear 1 / hDiffCorrFlux cubic
(system/fvSchemes:32-40), chemistry on with dfChemistryModel's default CVODE tolerances relTol 1e-9 /
absTol 1e-15 (constant/CanteraTorchProperties:22-25 leaves odeCoeffs empty; dfChemistryModel.C:57-58).
The reference samples T along x = z = 3 mm, y in [0, 6 mm] (1000 points, cellPoint; system/sample) at
t = 1e-4 .. 5e-4 s and test/corrtest.cpp:51-56 asserts five of those values (read at corrtest.cpp:20-24).

`lib_path` selects the implementation of include/dfmi.h: the HIP library (default) or the CPU-A baseline
(baseline/cpu_a/libdfmi_cpu_a.so), so the same driver pins both.
"""
from __future__ import annotations

import os

import numpy as np

L_TGV = 6.283185307179586e-3
# corrtest.cpp:20-24 (token k of postProcessing/sample/<t>/data_T.xy) and :52-56 (expected value)
TGV2D_EXPECTED = {100: (1100, 363.504), 200: (1064, 537.614), 300: (1064, 871.092), 400: (1098, 1297.64),
                  500: (806, 1532.92)}
SAMPLE_LINE = ((0.003, 0.0, 0.003), (0.003, 0.006, 0.003), 1000)   # system/sample: lineUniform axis y


def tgv2d_mesh():
    from .mesh import hex_box
    return hex_box(128, 128, 1, lengths=(L_TGV,) * 3, periodic=(True, True, False),
                   wall_kinds={"front": "empty", "back": "empty"})


def tgv2d_setup(case_dir: str, golden_dir: str, lib_path: str | None = None, chem_rtol=1e-9, chem_atol=1e-15,
                solver_tol=1e-10, schemes: dict | None = None, device: int = 0):
    """context + mesh with the case's initial state uploaded (createFields: thermo from T, phi, K)"""
    from .lib import Context
    from .mech import read_thermo_table, read_yaml_mechanism
    from .kinetics import parse_mechanism
    from .foam_io import read_case_fields
    from .schemes import read_fv_schemes
    from . import case
    yml = os.path.join(golden_dir, "ES80_H2-7-16.yaml")
    ym = read_yaml_mechanism(yml)
    sp = ym["species"]
    t = read_thermo_table(os.path.join(golden_dir, "thermo_ES80_H2-7-16.txt"), sp)
    m = tgv2d_mesh()
    if schemes is None:
        schemes = read_fv_schemes(os.path.join(case_dir, "fvSchemes"))
    ctx = Context(device, lib_path=lib_path)
    dt = 1e-6
    case.setup_context(ctx, m, t, sp.index("N2"), dt, schemes=schemes)
    ctx.chem_set_mechanism(parse_mechanism(yml))
    ctx.chem_set_options(1, rtol=chem_rtol, atol=chem_atol)
    ctx.chem_set_max_steps(1000000)
    for e in ("U", "Y", "E"):
        ctx.set_solver(e, 200, solver_tol, 1e-300)
    ctx.set_solver("p", 2000, solver_tol, 1e-300)
    f = read_case_fields(os.path.join(case_dir, "0"), sp)
    case.init_state(ctx, m, t.S, f["T"], f["p"], f["U"], f["Y"])
    return ctx, m, t, sp


def sample_T(m, T):
    from .sample import CellPointSampler
    s = CellPointSampler(m, m.nodes, (True, True, False))
    start, end, n = SAMPLE_LINE
    pts, vals = s.line_uniform(T, start, end, n)
    return pts[:, 1], vals


def corrtest_values(m, T, step):
    """the value test/corrtest.cpp reads for this step (token k of the raw set file)"""
    from .sample import raw_token_value
    y, v = sample_T(m, T)
    k, _ = TGV2D_EXPECTED[step]
    return raw_token_value(y, v, k), y, v


def run_tgv2d(case_dir: str, golden_dir: str, steps=500, lib_path=None, log=None, **kw):
    """500 outer iterations; -> {step: (value corrtest reads, expected, sampled line T)} at 100 .. 500"""
    ctx, m, t, sp = tgv2d_setup(case_dir, golden_dir, lib_path=lib_path, **kw)
    out = {}
    C = m.n_cells
    for n in range(1, steps + 1):
        ctx.time_step(2)
        if n in TGV2D_EXPECTED:
            T = ctx.get_field("T", (C,))
            val, y, v = corrtest_values(m, T, n)
            out[n] = {"value": val, "expected": TGV2D_EXPECTED[n][1], "T_max": float(T.max()),
                      "line_max": float(v.max()), "p_mean": float(ctx.get_field("p", (C,)).mean())}
            if log:
                log(f"step {n}: sampled T {val:.3f} K (corrtest {TGV2D_EXPECTED[n][1]}), line max {v.max():.3f}, "
                    f"cell max {T.max():.3f}")
    ctx.close()
    return out


# ------------------------------------------------------------------ 1D flame speed (test/Tu500K-Phi1)
# corrtest.cpp:269-270 asserts fs = 6 (token 3 of the fs file, corrtest.cpp:266,276-300): the third
# "flameSpeed = " line of applications/utilities/flameSpeed/flameSpeed.C:72 over the written times
# 0, 0.001, 0.002 (system/controlDict writeInterval 1e-3, endTime 2e-3) -> the speed between 1 and 2 ms.
FLAME_SPEED_EXPECTED = 6.0


def flame_position(m, T, bT, types_T):
    """flameSpeed.C:48-70: x of the cell centre with the largest x-gradient of T (fvc::grad, Gauss
    linear with T's boundary values; findMax = the first maximum)"""
    C = m.n_cells
    own, nei, w = m.owner, m.neighbour, m.weight
    fv = w * (T[own] - T[nei]) + T[nei]
    gx = np.zeros(C)
    np.add.at(gx, own, m.sf[:, 0] * fv)
    np.add.at(gx, nei, -m.sf[:, 0] * fv)
    off = 0
    for p, t in zip(m.patches, types_T):
        if p.kind != "empty" and p.size:
            np.add.at(gx, p.face_cells, p.sf[:, 0] * bT[off:off + p.size])
        off += p.slots
    gx /= m.volume
    return float(m.cell_centres[int(np.argmax(gx)), 0])


def run_flame1d_speed(golden_dir: str, steps=2000, lib_path=None, log=None, schemes: dict | None = None,
                      chem_rtol=1e-6, chem_atol=1e-10, solver_tol=1e-8, device: int = 0):
    """2 ms of the reference's 1D freely-propagating flame (880 cells, Burke2012, its 0/ fields, fvSchemes
    and waveTransmissive outlet; odeCoeffs relTol 1e-6 / absTol 1e-10) -> flame positions at 0, 1, 2 ms and
    the flameSpeed utility's value for the last interval"""
    from .lib import Context
    from .mech import read_thermo_table, read_yaml_mechanism
    from .kinetics import parse_mechanism
    from .schemes import read_fv_schemes
    from . import case
    fdir = os.path.join(golden_dir, "flame1d")
    yml = os.path.join(golden_dir, "Burke2012_s9r23.yaml")
    ym = read_yaml_mechanism(yml)
    t = read_thermo_table(os.path.join(golden_dir, "thermo_Burke2012_s9r23.txt"), ym["species"])
    m = case.flame1d_mesh()
    if schemes is None:
        schemes = read_fv_schemes(os.path.join(fdir, "fvSchemes"))
    ctx = Context(device, lib_path=lib_path)
    pt = case.flame1d_patch_types(m)
    case.setup_context(ctx, m, t, ym["species"].index("N2"), 1e-6, pt, schemes=schemes)
    ctx.chem_set_mechanism(parse_mechanism(yml))
    ctx.chem_set_options(1, rtol=chem_rtol, atol=chem_atol)
    for e in ("U", "Y", "E"):
        ctx.set_solver(e, 200, solver_tol, 1e-300)
    ctx.set_solver("p", 2000, solver_tol, 1e-300)
    f, bv = case.flame1d_fields(fdir, ym["species"])
    case.init_state(ctx, m, t.S, f["T"], f["p"], f["U"], f["Y"], bvals=bv, gammas=case.flame1d_gamma(fdir))
    U00 = float(f["U"][0, 0])   # flameSpeed.C:60-69 reads U from the 0 directory
    C, B = m.n_cells, m.n_boundary_slots

    def pos():
        return flame_position(m, ctx.get_field("T", (C,)), ctx.get_field("boundary_T", (B,)), pt["T"])
    xs = {0: pos()}
    for n in range(1, steps + 1):
        ctx.time_step(2)
        if n % 1000 == 0:
            xs[n] = pos()
            if log:
                log(f"step {n}: flame at x = {xs[n] * 1e3:.3f} mm")
    ctx.close()
    speeds = {}
    prev = 0.0211   # flameSpeed.C:37 initial flamePosition
    for n in sorted(xs):
        speeds[n] = U00 - (xs[n] - prev) / 0.001
        prev = xs[n]
    return {"positions": xs, "flameSpeed": speeds, "U_inlet": U00}
