"""Config 1 trajectory on the GPU at several integrator tolerances -> gpurun_out/zerod_traj.npz"""
import json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deepflame-dev_amd"))
from dfmi.mesh import hex_box
from dfmi.mech import read_thermo_table, read_yaml_mechanism
from dfmi.kinetics import parse_mechanism
from dfmi.lib import Context
from dfmi import case
golden = os.path.join(ROOT, "tests", "golden")
ref = json.load(open(os.path.join(golden, "zeroD_cubicReactor.json")))
ym = read_yaml_mechanism(os.path.join(golden, ref["mechanism"]))
t = read_thermo_table(os.path.join(golden, "thermo_ES80_H2-7-16.txt"), ym["species"])
out = {}
for tag, rtol, atol, generic in (("r10", 1e-10, 1e-20, 0), ("r12", 1e-12, 1e-22, 0), ("r10g", 1e-10, 1e-20, 1)):
    if generic:
        os.environ["DFMI_OPTIONS"] = "chem.generated=0"
    m = hex_box(2, 2, 2, lengths=(5e-3,) * 3, periodic=(False,) * 3)
    ctx = Context(0)
    case.setup_context(ctx, m, t, ym["species"].index("N2"), ref["dt"])
    ctx.chem_set_mechanism(parse_mechanism(os.path.join(golden, ref["mechanism"])))
    ctx.chem_set_options(1, rtol=rtol, atol=atol)
    C = m.n_cells
    case.init_state(ctx, m, t.S, np.full(C, ref["T0"]), np.full(C, ref["p"]), np.zeros((3, C)),
                    np.repeat(np.asarray(ref["Y0"])[:, None], C, axis=1))
    T = [ref["T0"]]
    steps = []
    for k in range(ref["n_steps"]):
        ctx.zero_d_step(ref["dt"], 1)
        T.append(ctx.get_field("T", (C,))[0])
        steps.append(ctx.get_field("chem_stats", (3, C))[:, 0])
    out[tag] = np.array(T)
    out[tag + "_stats"] = np.array(steps)
    ctx.close()
    os.environ.pop("DFMI_OPTIONS", None)
    print(tag, "T_end", T[-1], "max dT vs oracle", np.abs(np.array(T) - np.array(ref["T"])).max(), flush=True)
np.savez(os.path.join(ROOT, "gpurun_out", "zerod_traj.npz"), **out)
