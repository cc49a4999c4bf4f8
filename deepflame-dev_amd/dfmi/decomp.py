"""Host-side statement of the halo exchange plan (the lists halo.hip:halo_setup builds on the device
side), used by the multi-rank CPU tests and by tooling.

Per neighbour rank, the processor patches to it are concatenated in a canonical order both sides
derive independently: sorted by the (min, max) pair of global cell ids across the patch's first face.
Faces inside a patch keep OpenFOAM's matching order. The sender packs cell values of its
face cells; the receiver stores them in the neighbour half (first n slots) of its processor patches.
"""
from __future__ import annotations

import numpy as np

from .mesh import Mesh

PROC_KINDS = ("processor", "processorCyclic")


def halo_plan(m: Mesh) -> dict:
    """{peer: (send_cells, recv_slots)} in the canonical order (int64 arrays)."""
    offs, o = [], 0
    for p in m.patches:
        offs.append(o)
        o += p.slots
    by_peer = {}
    for pi, p in enumerate(m.patches):
        if p.kind not in PROC_KINDS:
            continue
        if p.size:
            a = m.global_offset + int(p.face_cells[0])
            b = int(p.nbr_cells_global[0])
            key = (min(a, b), max(a, b))
        else:
            key = (0, 0)
        by_peer.setdefault(p.peer_rank, []).append((key, pi))
    plan = {}
    for peer in sorted(by_peer):
        cells, slots = [], []
        for _, pi in sorted(by_peer[peer]):
            p = m.patches[pi]
            cells.append(p.face_cells.astype(np.int64))
            slots.append(offs[pi] + np.arange(p.size, dtype=np.int64))
        plan[peer] = (np.concatenate(cells), np.concatenate(slots))
    return plan


def exchange_numpy(plans: list, cell_fields: list, bnd_fields: list):
    """Single-process reference exchange over all ranks: cell_fields[r] is [k][C_r], bnd_fields[r]
    is [k][B_r] (updated in place)."""
    for r, plan in enumerate(plans):
        for peer, (cells, slots) in plan.items():
            src_cells, _ = plans[peer][r]
            bnd_fields[r][:, slots] = cell_fields[peer][:, src_cells]
