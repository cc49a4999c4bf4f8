"""The headline workload's own state (BASELINE config 3): a 32^3 tile of the reference example's 64^3 TGV
initial fields (examples/dfLowMachFoam/notorch/threeD_reactingTGV/H2/cvodeIntegrator/0, committed as
tests/golden/tgv64) around the hot kernel, Burke2012 9 species, with the stiff chemistry integrated
inside dfmi_time_step (mode 1, the reference CVODE tolerances).

- the GPU chemistry source of that state vs the oracle's SciPy-BDF integration on the hottest and on
  sampled cells (per-species scale, CVODE-level tolerance);
- one full outer iteration vs the oracle (exact solves) fed the same source: fields per component
  (per species) within 1e-9 relative.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, rel_err

pytestmark = pytest.mark.gpu


def test_tgv64_tile_with_chemistry_matches_oracle():
    from dfmi.mesh import hex_box
    from dfmi.mech import read_thermo_table, read_yaml_mechanism
    from dfmi.kinetics import parse_mechanism
    from dfmi.foam_io import read_case_fields
    from dfmi.lib import Context
    from dfmi import case
    import oracle as O
    from chem_oracle import Kinetics
    ym = read_yaml_mechanism(os.path.join(GOLDEN, "Burke2012_s9r23.yaml"))
    sp = ym["species"]
    t = read_thermo_table(os.path.join(GOLDEN, "thermo_Burke2012_s9r23.txt"), sp)
    mech = parse_mechanism(os.path.join(GOLDEN, "Burke2012_s9r23.yaml"))
    src = read_case_fields(os.path.join(GOLDEN, "tgv64"), sp)
    n, N = 32, 64
    hot = int(np.argmax(src["T"]))
    hi, hj, hk = hot % N, (hot // N) % N, hot // (N * N)
    o0 = [(v - n // 2) % N for v in (hi, hj, hk)]              # tile centred on the hottest cell
    m = hex_box(n, n, n, lengths=(2 * np.pi * 1e-3 * n / N,) * 3)
    ii, jj, kk = m.local_index
    idx = ((o0[0] + ii) % N) + N * (((o0[1] + jj) % N) + N * ((o0[2] + kk) % N))
    T0, p0 = src["T"][idx], src["p"][idx]
    U0, Y0 = np.ascontiguousarray(src["U"][:, idx]), np.ascontiguousarray(src["Y"][:, idx])
    assert T0.max() > 1800.0
    ctx = Context(0)
    inert = sp.index("N2")
    dt = 1e-6
    pt = case.setup_context(ctx, m, t, inert, dt)
    ctx.chem_set_mechanism(mech)
    ctx.chem_set_options(1, rtol=1e-6, atol=1e-10)
    case.init_state(ctx, m, t.S, T0, p0, U0, Y0)
    st = case.pull_state(ctx, m, t.S)
    C = m.n_cells
    # the chemistry source of this state, as the time step will compute it (same T, p, Y, rho = rho_old)
    ctx.set_field("chem_stats", np.zeros((3, C)))
    ctx.chem_solve(dt)
    RR = ctx.get_field("RR", (t.S, C))
    # ... against the oracle's BDF integration on the hottest cells and a spread sample
    order = np.argsort(st["T"])
    sel = np.unique(np.concatenate([order[-24:], order[:: C // 24]]))
    kin = Kinetics(mech, ym["nasa"], ym["W"])
    print(f"tile {n}^3: GPU chemistry done, oracle BDF on {sel.size} cells", flush=True)
    ref = kin.reaction_rates(st["T"][sel], st["p"][sel], st["rho"][sel], st["Y"][:, sel], dt, rtol=1e-10, atol=1e-20)
    scale = np.maximum(np.abs(ref).max(axis=1, keepdims=True), 1e-3 * np.abs(ref).max())
    assert np.abs(RR).max() > 0
    assert (np.abs(RR[:, sel] - ref) / scale).max() < 2e-3
    # heat release Qdot = -sum_i hc_i RR_i of that source (dfChemistryModel.C:771) vs the oracle's sum
    from chem_oracle import heat_release, hf298_per_mass
    q = ctx.get_field("Qdot", (C,))
    qref = heat_release(hf298_per_mass(t.nasa, t.W), RR)
    assert rel_err(q, qref) <= 1e-12, rel_err(q, qref)
    assert q.max() > 0
    assert (np.abs(heat_release(hf298_per_mass(t.nasa, t.W), ref) - q[sel]) / np.abs(qref).max()).max() < 2e-3
    # one outer iteration with the chemistry inside the step vs the oracle fed the same source
    case.push_state(ctx, st)
    ctx.set_field("chem_stats", np.zeros((3, C)))
    for e in ("U", "Y", "E"):
        ctx.set_solver(e, 300, 1e-15, 1e-300)
    ctx.set_solver("p", 3000, 1e-15, 1e-300)
    ctx.call("pre_time_step")
    st2 = dict(st)
    ctx.time_step(2)
    assert np.array_equal(ctx.get_field("RR", (t.S, C)), RR)   # the step integrated exactly that source
    assert np.array_equal(ctx.get_field("Qdot", (C,)), q)       # ... and reported its heat release
    st2["RR"] = RR
    print("GPU step done, oracle step", flush=True)
    o = O.Oracle(m, t, {k: v.copy() for k, v in st2.items()}, pt, inert, 1.0 / dt)
    o.time_step(2)
    print("oracle step done", flush=True)
    for nme, tl in {"T": 1e-10, "p": 1e-11, "rho": 1e-10, "he": 1e-10}.items():
        e = rel_err(ctx.get_field(nme, (C,)), o[nme])
        assert e < tl, (nme, e)
    assert rel_err(ctx.get_field("U", (3, C)), o["U"]) < 1e-9
    assert rel_err(ctx.get_field("Y", (t.S, C)), o["Y"]) < 1e-9
    assert rel_err(ctx.get_field("phi", (m.n_faces,)), o["phi"]) < 1e-9
    ctx.close()
