"""Decomposed-AMG iteration growth: the pressure PCG's AMG aggregates stop at rank
boundaries (block-Jacobi across processor faces), so more ranks can mean more PCG iterations. On one GPU,
R = 1, 2, 4, 8 in-process ranks (dfmi_set_comm_local: the code path RCCL runs, halo messages as device
copies) split an n^3 periodic box (the reference TGV fields tiled, Burke 9 species, chemistry off) as
decomposePar blocks; each configuration runs a few outer iterations with the production solver controls
and reports the p-solve iterations. Prints one JSON line per R.

Usage: python scripts/amg_decomp_study.py [n=64] [steps=4] [strong|weak]
(strong: one n^3 box split R ways; weak: an n^3 block per rank, the bench's --gpus N layout)"""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deepflame-dev_amd"))
sys.path.insert(0, ROOT)


def run(n, decomp, steps, hub, weak=False):
    import numpy as np
    from bench import MECHS, reference_fields
    from dfmi.mesh import hex_box
    from dfmi.mech import read_thermo_table, read_yaml_mechanism
    from dfmi.lib import Context
    from dfmi import case
    g = os.path.join(ROOT, "tests", "golden")
    ym = read_yaml_mechanism(os.path.join(g, MECHS["burke9"][0]))
    t = read_thermo_table(os.path.join(g, MECHS["burke9"][1]), ym["species"])
    L = 2 * np.pi * 1e-3
    nr = int(np.prod(decomp))
    out, err = [None] * nr, [None] * nr

    def work(r):
        try:
            if weak:
                m = hex_box(n * decomp[0], n * decomp[1], n * decomp[2], lengths=(L * decomp[0], L * decomp[1], L * decomp[2]),
                            decomp=decomp, rank=r)
            else:
                m = hex_box(n, n, n, lengths=(L, L, L), decomp=decomp, rank=r)
            ctx = Context(0)
            comm = {"hub": hub, "nranks": nr, "rank": r} if nr > 1 else None
            case.setup_context(ctx, m, t, ym["species"].index("N2"), 1e-6, comm=comm)
            f = reference_fields(m, ym["species"])
            case.init_state(ctx, m, t.S, f["T"], f["p"], f["U"], f["Y"])
            ctx.time_step(2)
            ctx.solver_work("p", reset=True)
            t0 = time.perf_counter()
            iters = []
            for _ in range(steps):
                ctx.time_step(2)
                iters.append(ctx.solver_stats("p")[0])
            ctx.sync()
            el = time.perf_counter() - t0
            out[r] = {"p_iters_last_solve": iters, "p_iters_per_step": ctx.solver_work("p") / steps,
                      "ms_per_step": el / steps * 1e3, "amg_levels": ctx.amg_info()}
            ctx.close()
        except Exception as e:
            err[r] = e

    th = [threading.Thread(target=work, args=(r,)) for r in range(nr)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=240)
    if any(x.is_alive() for x in th):
        raise RuntimeError("decomposed run hung")
    for e in err:
        if e is not None:
            raise e
    return out[0]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    weak = len(sys.argv) > 3 and sys.argv[3] == "weak"
    for i, decomp in enumerate([(1, 1, 1), (2, 1, 1), (2, 2, 1), (2, 2, 2)]):
        r = run(n, decomp, steps, 900 + i, weak)
        R = int(decomp[0] * decomp[1] * decomp[2])
        print(json.dumps({"ranks": R, "decomp": decomp, "mode": "weak" if weak else "strong",
                          "global_cells": n ** 3 * (R if weak else 1), **r}), flush=True)


if __name__ == "__main__":
    main()
