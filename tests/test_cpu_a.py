"""CPU-A: the OpenMP C++ CPU implementation of the step behind include/dfmi.h
(baseline/cpu_a) that bench.py's cpu_baseline leg times. Runs on the CPU: it exports the whole ABI,
one outer iteration with tight solves equals the oracle's (exact solves), its ROS3 chemistry matches the
SciPy-BDF restatement, and the default AMG-PCG / BiCGStab controls converge."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, rel_err

CPU_A = os.path.join(ROOT, "baseline", "cpu_a", "libdfmi_cpu_a.so")


def _ctx():
    from dfmi.lib import Context
    if not os.path.exists(CPU_A):
        pytest.fail("CPU-A library not built (make -C baseline/cpu_a)")
    return Context(0, lib_path=CPU_A)


def _mech():
    from dfmi.mech import read_thermo_table, read_yaml_mechanism
    from dfmi.kinetics import parse_mechanism
    ym = read_yaml_mechanism(os.path.join(GOLDEN, "Burke2012_s9r23.yaml"))
    t = read_thermo_table(os.path.join(GOLDEN, "thermo_Burke2012_s9r23.txt"), ym["species"])
    return ym, t, parse_mechanism(os.path.join(GOLDEN, "Burke2012_s9r23.yaml"))


def _case(walls):
    from dfmi import case
    from dfmi.mesh import (hex_box, FIXED_VALUE, FIXED_ENERGY, GRADIENT_ENERGY, INLET_OUTLET, WAVE_TRANSMISSIVE)
    ym, t, mech = _mech()
    L = 2 * np.pi * 1e-3
    m = hex_box(8, 6, 5, lengths=(L,) * 3, periodic=(not walls,) * 3, gradings=(1.0, 1.4, 1.0))
    pt = case.default_patch_types(m)
    refs = gammas = None
    if walls:   # inlet on "left", an open outlet (inletOutlet U/Y, waveTransmissive p) on "right"
        left = [i for i, p in enumerate(m.patches) if p.name == "left"]
        right = [i for i, p in enumerate(m.patches) if p.name == "right"]
        for f in ("U", "T", "Y"):
            pt[f] = m.patch_types(0).copy(); pt[f][left] = FIXED_VALUE
        pt["he"] = m.patch_types(GRADIENT_ENERGY).copy(); pt["he"][left] = FIXED_ENERGY
        pt["U"][right] = INLET_OUTLET; pt["Y"][right] = INLET_OUTLET
        pt["p"] = m.patch_types(0).copy(); pt["p"][right] = WAVE_TRANSMISSIVE
        yu, _ = case.h2_air_compositions(ym["species"])
        refs = {"U": {"right": np.array([0.3, -0.1, 0.2])}, "Y": {"right": yu}}
        gammas = {"right": 1.4}
    ctx = _ctx()
    inert = ym["species"].index("N2")
    dt = 1e-6
    case.setup_context(ctx, m, t, inert, dt, pt)
    f = case.tgv_fields(m, ym["species"], kernel_radius=1.2e-3)
    case.init_state(ctx, m, t.S, f["T"], f["p"], f["U"], f["Y"], refs=refs, gammas=gammas)
    ctx.call("pre_time_step")
    rng = np.random.default_rng(7)
    st = case.pull_state(ctx, m, t.S)
    st["rho_old"] = st["rho"] * (1 + 1e-3 * rng.standard_normal(m.n_cells))
    st["RR"] = 1e2 * rng.standard_normal((t.S, m.n_cells))
    st["dpdt"] = 1e3 * rng.standard_normal(m.n_cells)
    case.push_state(ctx, st)
    return ctx, m, t, st, pt, inert, dt, ym, mech


def test_exports_every_header_symbol():
    import ctypes
    import re
    hdr = open(os.path.join(ROOT, "include", "dfmi.h")).read()
    names = set(re.findall(r"\b(dfmi_\w+)\s*\(", hdr))
    lib = ctypes.CDLL(CPU_A)
    missing = [n for n in sorted(names) if not hasattr(lib, n)]
    assert not missing, missing
    lib.dfmi_version.restype = ctypes.c_char_p
    assert b"CPU-A" in lib.dfmi_version()


@pytest.mark.parametrize("walls", [False, True], ids=["periodic", "open-outlet"])
def test_outer_iteration_matches_oracle(walls):
    import oracle as O
    ctx, m, t, st, pt, inert, dt, ym, mech = _case(walls)
    for e in ("U", "Y", "E"):
        ctx.set_solver(e, 300, 1e-15, 1e-300)
    ctx.set_solver("p", 3000, 1e-15, 1e-300)
    o = O.Oracle(m, t, {k: v.copy() for k, v in st.items()}, pt, inert, 1.0 / dt)
    o.time_step(2)
    ctx.time_step(2)
    for n, tl in {"T": 1e-10, "p": 1e-11, "rho": 1e-10, "he": 1e-10}.items():
        assert rel_err(ctx.get_field(n, (m.n_cells,)), o[n]) < tl, n
    assert rel_err(ctx.get_field("U", (3, m.n_cells)), o["U"]) < 1e-9
    assert rel_err(ctx.get_field("Y", (t.S, m.n_cells)), o["Y"]) < 1e-9
    assert rel_err(ctx.get_field("phi", (m.n_faces,)), o["phi"]) < 1e-9
    B = m.n_boundary_slots
    assert rel_err(ctx.get_field("boundary_p", (B,)), o["boundary_p"]) < 1e-9


def test_default_solvers_converge_and_amg_beats_jacobi():
    ctx, m, t, st, pt, inert, dt, ym, mech = _case(False)
    ctx.time_step(2)
    it_amg, r0, rel = ctx.solver_stats("p")
    assert rel <= 1e-5 and it_amg > 0
    for e in ("U", "Y", "E"):
        it, r0, rel = ctx.solver_stats(e)
        assert rel <= 1e-5 and 0 < it < 20, (e, it, rel)   # converged inside the AmgX limit (amgxUOptions: 20)
    from dfmi import case
    case.push_state(ctx, st)
    ctx.set_preconditioner("p", "jacobi")
    ctx.time_step(2)
    it_jac, _, _ = ctx.solver_stats("p")
    assert it_amg < it_jac


def test_chemistry_matches_bdf():
    from chem_oracle import Kinetics
    ctx, m, t, st, pt, inert, dt, ym, mech = _case(False)
    ctx.chem_set_mechanism(mech)
    ctx.chem_set_options(1, rtol=1e-8, atol=1e-14)
    assert ctx.chem_info() == 1           # the compiled-in Burke mechanism
    ctx.chem_solve(dt)
    T = ctx.get_field("T", (m.n_cells,))
    p = ctx.get_field("p", (m.n_cells,))
    rho = ctx.get_field("rho", (m.n_cells,))
    Y = ctx.get_field("Y", (t.S, m.n_cells))
    idx = np.argsort(T)[-24:]             # the hot kernel: the reacting cells
    rr = ctx.get_field("RR", (t.S, m.n_cells))[:, idx]
    ref = Kinetics(mech, ym["nasa"], ym["W"]).reaction_rates(T[idx], p[idx], rho[idx], Y[:, idx], dt)
    scale = np.maximum(np.abs(ref).max(axis=1, keepdims=True), 1e-3 * np.abs(ref).max())
    assert np.abs(ref).max() > 0
    assert (np.abs(rr - ref) / scale).max() < 1e-4


def test_zero_d_steps_follow_the_oracle_trajectory():
    """BASELINE config 1 on CPU-A (dfmi_zero_d_step): the df0DFoam reactor of the reference example
    against the committed oracle trajectory (tests/golden/zeroD_cubicReactor.json)"""
    import json
    from dfmi import case
    from dfmi.mesh import hex_box
    from dfmi.mech import read_thermo_table, read_yaml_mechanism
    from dfmi.kinetics import parse_mechanism
    ref = json.load(open(os.path.join(GOLDEN, "zeroD_cubicReactor.json")))
    ym = read_yaml_mechanism(os.path.join(GOLDEN, ref["mechanism"]))
    t = read_thermo_table(os.path.join(GOLDEN, "thermo_ES80_H2-7-16.txt"), ym["species"])
    m = hex_box(3, 3, 3, lengths=(5e-3,) * 3, periodic=(False,) * 3)
    ctx = _ctx()
    case.setup_context(ctx, m, t, ym["species"].index("N2"), ref["dt"])
    ctx.chem_set_mechanism(parse_mechanism(os.path.join(GOLDEN, ref["mechanism"])))
    ctx.chem_set_options(1, rtol=1e-12, atol=1e-22)   # the fixture's converged trajectory (test_gpu_zero_d)
    C = m.n_cells
    case.init_state(ctx, m, t.S, np.full(C, ref["T0"]), np.full(C, ref["p"]), np.zeros((3, C)),
                    np.repeat(np.asarray(ref["Y0"])[:, None], C, axis=1))
    n = min(300, ref["n_steps"])
    ctx.zero_d_step(ref["dt"], n)
    T = ctx.get_field("T", (C,))
    assert np.ptp(T) <= 1e-12 * T[0]
    assert abs(T[0] - ref["T"][n]) <= 2e-5 * ref["T"][n]
