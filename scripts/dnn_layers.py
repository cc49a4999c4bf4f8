"""DF-ODENet GEMM timing on BASELINE config 4's 53-species nets [55, 1600, 800, 400, 1] (seeded weights): every
cell of an n^3 mesh reacting, HIP-event timers around the GEMM launches. One JSON line: wall ms per
inference, GEMM ms per 65,536-row chunk and TFLOP/s. Usage: python scripts/dnn_layers.py [n=64] [reps=3]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deepflame-dev_amd"))


def main():
    import torch  # noqa: F401  (HIP runtime first)
    from dfmi import case, dnn_model
    from dfmi.lib import Context
    from dfmi.mesh import hex_box
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    S = 53
    m = hex_box(n, n, n)
    C = m.n_cells
    rng = np.random.default_rng(0)
    Y = rng.gamma(0.3, 1.0, (S, C))
    Y /= Y.sum(axis=0)
    T = np.full(C, 1500.0)
    p = np.full(C, 101325.0)
    Wm = 1.0 / (Y / np.linspace(2.0, 44.0, S)[:, None]).sum(axis=0)
    rho = p * Wm / (8314.46261815324 * T)
    ctx = Context(0)
    pt = case.default_patch_types(m)
    rows, cols = m.proc_rows_cols()
    ctx.set_constant_values(C, C, m.n_faces, m.n_boundary_slots, m.n_patches, int(rows.size), m.patch_sizes, S, 1e6)
    ctx.set_cyclic_info(m.cyclic_neighbour())
    ctx.set_constant_indexes(m.owner, m.neighbour, rows, cols, 0)
    ctx.init_constant_fields_internal(m.sf, m.mag_sf, m.weight, m.delta_coeffs, m.volume, m.mesh_distance)
    bsf, bmag, bdc, bw, bfc = m.boundary_arrays()
    ctx.init_constant_fields_boundary(bsf, bmag, bdc, bw, bfc, pt["calculated"], pt["extrapolated"])
    ctx.set_inert_index(S - 1)
    dims = [int(v) for v in os.environ["DIMS"].split(",")] if os.environ.get("DIMS") else [S + 2, 1600, 800, 400, 1]
    ctx.dnn_set_model(dims, dnn_model.seeded_weights(n_modules=S - 1, dims=dims), np.zeros(S + 2), np.ones(S + 2),
                      np.zeros(S - 1), np.full(S - 1, 0.01))
    ctx.chem_set_options(2)
    for k, v in (("T", T), ("p", p), ("rho", rho), ("Y", Y)):
        ctx.set_field(k, v)
    ctx.dnn_infer()
    ctx.kernel_timer("k_mlp_gemm")
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        nr = ctx.dnn_infer()
    el = time.perf_counter() - t0
    chunks = reps * ((nr + 65535) // 65536)
    nm = S - 1
    flops = [2.0 * nr * nm * dims[l] * dims[l + 1] for l in range(3)]
    flops[2] += 2.0 * nr * nm * dims[3]
    ms, launches = ctx.kernel_time("k_mlp_gemm")
    out = {"rows": nr, "ms_per_inference": el / reps * 1e3, "gemm_ms_per_chunk": ms / chunks, "launches": launches,
           "gemm_tflops": sum(flops) * reps / (ms / 1e3) / 1e12}
    ctx.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
