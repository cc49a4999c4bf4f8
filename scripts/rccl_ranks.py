"""Decomposed dfLowMachFoam step over the RCCL transport, one process per rank (torchrun worker).

The pool's GPU boxes have one MI355X and RCCL refuses two ranks on one device ("Duplicate GPU
detected": the check compares the host hash and the PCI bus id). Each rank therefore sets its own
NCCL_HOSTID before RCCL initialises: the ranks look like two hosts, so RCCL connects them through its
network transport (sockets over loopback) instead of P2P/xGMI. Everything above the wire is the
product path the 8-GPU run takes: ncclCommInitRank from a unique id, one ncclSend/ncclRecv group per
exchange point, ncclAllGather of the per-rank partial sums, the comm stream of the overlapped halos.

Rank 0 gathers the fields (through files), runs the undecomposed mesh on the same GPU and the oracle
(--no-oracle for meshes beyond its reach), and writes the relative errors to --out (JSON). Launched by
tests/test_gpu_rccl.py and, at BASELINE config 5's size (256^3 = 16.8M cells, 8 ranks 2x2x2), by
scripts/rccl_config5.sh:
  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P \
      scripts/rccl_ranks.py --decomp 2,1,1 --out gpurun_out/rccl.json
"""
import argparse
import json
import os
import sys

RANK = int(os.environ.get("RANK", "0"))
WORLD = int(os.environ.get("WORLD_SIZE", "1"))
# before anything loads RCCL: one "host" per rank, sockets over loopback, no InfiniBand probing
os.environ["NCCL_HOSTID"] = f"dfmi-rccl-rank{RANK}"
os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
os.environ.setdefault("NCCL_IB_DISABLE", "1")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "deepflame-dev_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np                      # noqa: E402
import torch.distributed as dist        # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--decomp", default="2,1,1")
    ap.add_argument("--mesh", default="10,8,6")
    ap.add_argument("--overlap", type=int, default=0)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--walls", type=int, default=0)
    ap.add_argument("--out", default="gpurun_out/rccl.json")
    ap.add_argument("--no-oracle", action="store_true", help="skip the oracle (meshes too large for it)")
    ap.add_argument("--tol", type=float, default=1e-14, help="relative solver tolerance of every equation")
    a = ap.parse_args()
    decomp = tuple(int(x) for x in a.decomp.split(","))
    nx, ny, nz = (int(x) for x in a.mesh.split(","))
    assert int(np.prod(decomp)) == WORLD, "decomposition must have WORLD_SIZE blocks"
    os.environ["DFMI_HALO_OVERLAP"] = str(a.overlap)

    dist.init_process_group("gloo", rank=RANK, world_size=WORLD)
    from dfmi.lib import Context
    from dfmi.mesh import hex_box, global_cell_ids
    from dfmi.mech import read_thermo_table, read_yaml_mechanism
    from dfmi import case
    from conftest import GOLDEN, rel_err

    ym = read_yaml_mechanism(os.path.join(GOLDEN, "ES80_H2-7-16.yaml"))
    t = read_thermo_table(os.path.join(GOLDEN, "thermo_ES80_H2-7-16.txt"), ym["species"])
    inert = ym["species"].index("N2")
    L = (2 * np.pi * 1e-3,) * 3
    dt = 1e-6
    periodic = (not a.walls,) * 3
    grad = (1.0, 1.3, 1.0)
    # the undecomposed mesh only on rank 0 (its reference run); every rank's initial state is the same
    # analytic TGV field evaluated at its own cell centres
    mg = hex_box(nx, ny, nz, lengths=L, gradings=grad, periodic=periodic) if RANK == 0 else None

    def setup(m, comm=None):
        ctx = Context(0)
        case.setup_context(ctx, m, t, inert, dt, case.default_patch_types(m), comm=comm)
        for e in ("U", "Y", "E"):
            ctx.set_solver(e, 300, a.tol, 1e-300)
        ctx.set_solver("p", 3000, a.tol, 1e-300)
        return ctx

    def fields(ctx, n):
        o = {k: ctx.get_field(k, (n,)) for k in ("T", "p", "rho", "he")}
        o["U"] = ctx.get_field("U", (3, n))
        o["Y"] = ctx.get_field("Y", (t.S, n))
        return o

    m = hex_box(nx, ny, nz, lengths=L, gradings=grad, periodic=periodic, decomp=decomp, rank=RANK)
    g = global_cell_ids(m, nx, ny)
    uid = [Context.unique_id() if RANK == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    c = setup(m, comm={"uid": uid[0], "nranks": WORLD, "rank": RANK})
    fl = case.tgv_fields(m, ym["species"], kernel_radius=1.2e-3)
    case.init_state(c, m, t.S, fl["T"], fl["p"], fl["U"], fl["Y"])
    del fl
    c.call("pre_time_step")
    c.comm_timer(True)   # transport calls and bytes per exchange point (the side stream's listed as "@side")
    for _ in range(a.steps):
        c.time_step(2)
    mine = fields(c, m.n_cells)
    mine["gid"] = g
    mine["p_iters"] = int(c.solver_stats("p")[0])
    comm = c.comm_report()
    c.comm_timer(False)
    c.close()
    every_comm = [None] * WORLD
    dist.all_gather_object(every_comm, {k: {"calls": v["calls"], "bytes": v["bytes"]} for k, v in comm.items()})
    # fields travel through files (a 16M-cell run would push GBs through the object collectives)
    import tempfile
    xdir = [tempfile.mkdtemp(prefix="dfmi_rccl_") if RANK == 0 else None]
    dist.broadcast_object_list(xdir, src=0)
    np.savez(os.path.join(xdir[0], f"rank{RANK}.npz"), **{k: np.asarray(v) for k, v in mine.items()})
    del mine
    dist.barrier()
    if RANK == 0:
        allr = [dict(np.load(os.path.join(xdir[0], f"rank{r}.npz"))) for r in range(WORLD)]
        glob = {}
        for n, k in (("T", 1), ("p", 1), ("rho", 1), ("he", 1), ("U", 3), ("Y", t.S)):
            arr = np.zeros((k, mg.n_cells))
            for o in allr:
                arr[:, o["gid"]] = o[n].reshape(k, -1)
            glob[n] = arr.reshape(-1, mg.n_cells) if k > 1 else arr[0]
        ref_ctx = setup(mg)
        f = case.tgv_fields(mg, ym["species"], kernel_radius=1.2e-3)
        case.init_state(ref_ctx, mg, t.S, f["T"], f["p"], f["U"], f["Y"])
        del f
        ref_ctx.call("pre_time_step")
        res = {"world": WORLD, "decomp": list(decomp), "mesh": [nx, ny, nz], "cells": mg.n_cells,
               "overlap": a.overlap, "steps": a.steps, "tol": a.tol,
               "p_iters_per_rank": [int(o["p_iters"]) for o in allr], "vs_single_domain": {}, "vs_oracle": {}}
        pts = sorted({k for e in every_comm for k in e})
        res["comm_per_step"] = {k: {"calls_max": max(e.get(k, {}).get("calls", 0) for e in every_comm) / a.steps,
                                    "bytes_max": max(e.get(k, {}).get("bytes", 0.0) for e in every_comm) / a.steps}
                                for k in pts}
        res["comm_calls_per_step_max"] = max(sum(v["calls"] for v in e.values()) for e in every_comm) / a.steps
        res["comm_bytes_per_step_max"] = max(sum(v["bytes"] for v in e.values()) for e in every_comm) / a.steps
        orc = None
        if a.steps == 1 and not a.no_oracle:
            import oracle as O
            st = case.pull_state(ref_ctx, mg, t.S)
            orc = O.Oracle(mg, t, {k: v.copy() for k, v in st.items()}, case.default_patch_types(mg), inert, 1.0 / dt)
            orc.time_step(2)
        for _ in range(a.steps):
            ref_ctx.time_step(2)
        ref = fields(ref_ctx, mg.n_cells)
        ref_ctx.close()
        for n in ("T", "p", "rho", "he", "U", "Y"):
            res["vs_single_domain"][n] = float(rel_err(glob[n], ref[n]))
            if orc is not None:
                res["vs_oracle"][n] = float(rel_err(glob[n], orc[n]))
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as fh:
            json.dump(res, fh, indent=1)
        print(json.dumps(res), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
