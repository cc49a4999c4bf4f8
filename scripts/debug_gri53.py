"""Config 4 (53 species, DNN) on a small box: per-stage field statistics to find where a step goes wrong."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deepflame-dev_amd"))
from dfmi.mesh import hex_box
from dfmi.mech import read_thermo_table
from dfmi.lib import Context
from dfmi import case
from dfmi.synthetic import gri53_species, gri53_smooth_fractions, gri53_dnn

golden = os.path.join(ROOT, "tests", "golden")
sp = gri53_species(os.path.join(golden, "gri30.yaml"))
t = read_thermo_table(os.path.join(golden, "thermo_gri53_synthetic.txt"), sp)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
m = hex_box(n, n, n)
ctx = Context(0)
case.setup_context(ctx, m, t, sp.index("N2"), 1e-6)
mode = sys.argv[2] if len(sys.argv) > 2 else "dnn"
if mode == "dnn":
    gri53_dnn(ctx)
    ctx.chem_set_options(2)
f = case.tgv_fields(m, ["H2", "O2", "N2", "H2O"], kernel_radius=1.5e-3)
C = m.n_cells
case.init_state(ctx, m, t.S, f["T"], f["p"], f["U"], gri53_smooth_fractions((f["T"] - 300.0) / np.ptp(f["T"])))


def stats(tag):
    out = [tag]
    for nme, shp in (("T", (C,)), ("p", (C,)), ("rho", (C,)), ("he", (C,)), ("U", (3, C)), ("Y", (t.S, C)),
                     ("RR", (t.S, C)), ("rhoD", (t.S, C)), ("mu", (C,)), ("alpha", (C,))):
        a = ctx.get_field(nme, shp)
        out.append(f"{nme}[{np.nanmin(a):.3g},{np.nanmax(a):.3g}{'' if np.isfinite(a).all() else ' NaN!'}]")
    print(" ".join(out), flush=True)


stats("init")
ctx.call("pre_time_step")
for step in range(3):
    for stage in ("rho_process", "U_process", "Y_process", "E_process", "thermo_correct"):
        ctx.call(stage)
        stats(f"step{step} {stage}")
        print("   iters", {e: ctx.solver_stats(e) for e in ("U", "Y", "E") if stage.startswith(e) or stage == "thermo_correct"}, flush=True)
    for _ in range(2):
        for stage in ("thermo_update_rho", "thermo_psip0", "U_get_HbyA", "p_process", "thermo_correct_psip_rho", "rho_process"):
            ctx.call(stage)
        stats(f"step{step} pcorr")
        print("   p iters", ctx.solver_stats("p"), flush=True)
    ctx.call("thermo_update_rho")
    ctx.call("pre_time_step")
