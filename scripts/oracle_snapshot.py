"""Run the oracle's stages on host-built states (periodic box, walled box with mixed BCs) and save every
array to an .npz -- used to check that restructuring the oracle (e.g. its OpenMP gathers) leaves its
results bitwise unchanged. Usage: python scripts/oracle_snapshot.py out.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deepflame-dev_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)


def run(tag, m, pt, out):
    import oracle as O
    from bench import host_state, MECHS
    from dfmi.mech import read_thermo_table, read_yaml_mechanism
    from dfmi import case
    g = os.path.join(ROOT, "tests", "golden")
    ym = read_yaml_mechanism(os.path.join(g, MECHS["burke9"][0]))
    t = read_thermo_table(os.path.join(g, MECHS["burke9"][1]), ym["species"])
    f = case.tgv_fields(m, ym["species"], kernel_radius=1.2e-3)
    st = host_state(m, t, f)
    rng = np.random.default_rng(7)
    st["rho_old"] = st["rho"] * (1 + 1e-3 * rng.standard_normal(m.n_cells))
    st["RR"] = 1e2 * rng.standard_normal((t.S, m.n_cells))
    B = m.n_boundary_slots
    st["boundary_p_gamma"] = np.full(B, 1.4)
    st["boundary_p_vf"] = np.zeros(B)
    st["boundary_U_ref"] = np.tile(np.array([0.3, -0.1, 0.2])[:, None], (1, B))
    st["boundary_Y_ref"] = np.tile(st["Y"][:, :1], (1, B))
    o = O.Oracle(m, t, {k: v.copy() for k, v in st.items()}, pt, ym["species"].index("N2"), 1e6)
    o.time_step(2)
    for k, v in o.arr.items():
        out[tag + "/" + k] = v.copy()


def main():
    from dfmi.mesh import hex_box, FIXED_VALUE, FIXED_ENERGY, GRADIENT_ENERGY, INLET_OUTLET, WAVE_TRANSMISSIVE
    from dfmi import case
    out = {}
    m = hex_box(8, 6, 5, lengths=(2 * np.pi * 1e-3,) * 3, gradings=(1.0, 1.4, 1.0))
    run("periodic", m, case.default_patch_types(m), out)
    m = hex_box(8, 6, 5, lengths=(2 * np.pi * 1e-3,) * 3, periodic=(False,) * 3, gradings=(1.0, 1.4, 1.0))
    pt = case.default_patch_types(m)
    left = [i for i, p in enumerate(m.patches) if p.name == "left"]
    right = [i for i, p in enumerate(m.patches) if p.name == "right"]
    for fld in ("U", "T", "Y"):
        pt[fld] = m.patch_types(0).copy(); pt[fld][left] = FIXED_VALUE
    pt["he"] = m.patch_types(GRADIENT_ENERGY).copy(); pt["he"][left] = FIXED_ENERGY
    pt["U"][right] = INLET_OUTLET; pt["Y"][right] = INLET_OUTLET
    pt["p"] = m.patch_types(0).copy(); pt["p"][right] = WAVE_TRANSMISSIVE
    run("walls", m, pt, out)
    np.savez(sys.argv[1], **out)
    print(len(out), "arrays")


if __name__ == "__main__":
    main()
