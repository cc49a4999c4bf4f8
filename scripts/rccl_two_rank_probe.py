"""Probe: two ranks on ONE GPU through the RCCL transport (torchrun --nproc-per-node 2).
RCCL normally refuses two ranks per device; if it does, this prints the error and exits 0."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deepflame-dev_amd"))
import numpy as np
import torch
import torch.distributed as dist

rank = int(os.environ["RANK"]); world = int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", rank=rank, world_size=world)
from dfmi.mesh import hex_box
from dfmi.mech import read_thermo_table, read_yaml_mechanism
from dfmi.lib import Context, DfmiError
from dfmi import case
g = os.path.join(ROOT, "tests", "golden")
ym = read_yaml_mechanism(os.path.join(g, "Burke2012_s9r23.yaml"))
t = read_thermo_table(os.path.join(g, "thermo_Burke2012_s9r23.txt"), ym["species"])
m = hex_box(16, 8, 8, decomp=(2, 1, 1), rank=rank)
ctx = Context(0)
uid = [Context.unique_id() if rank == 0 else None]
dist.broadcast_object_list(uid, src=0)
try:
    case.setup_context(ctx, m, t, 8, 1e-6, comm={"uid": uid[0], "nranks": world, "rank": rank})
except DfmiError as e:
    print(f"rank {rank}: RCCL setup refused: {e}", flush=True)
    sys.exit(0)
f = case.tgv_fields(m, ym["species"])
case.init_state(ctx, m, t.S, f["T"], f["p"], f["U"], f["Y"])
ctx.call("pre_time_step")
ctx.time_step(2)
T = ctx.get_field("T", (m.n_cells,))
print(f"rank {rank}: RCCL two-rank step ok, T in [{T.min():.1f}, {T.max():.1f}], p iters {ctx.solver_stats('p')[0]}",
      flush=True)
dist.destroy_process_group()
