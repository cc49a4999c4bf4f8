"""DF-ODENet surrogate (A9) on MI355X vs a plain PyTorch fp32 restatement of the reference's
inference (dfChemistrySolver.cu:4-75 pre/post-processing; inference.py:12-25 NN_MLP).
The model weights of the reference are not in the repository: nets are seeded
N(0, 1/fan_in). Inference runs in fp16 with fp32 accumulation, like the reference's .to(kHalf)
modules, so RR is compared at 2e-2 of each species' scale (fp16 has an 11-bit mantissa)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

# normalisation constants the reference hard-codes for its H2 9-species nets (dfChemistrySolver.cu:95-105)
XMU = [1.2996375154e+03, 1.4349643303e+05, -4.3678815323e+00, -5.8949183472e+00, -3.8840763486e+00,
       -5.5436246211e+00, -6.0178199636e+00, -2.1469850084e+00, -6.9828365432e+00, -7.7747568654e+00,
       -1.8571483828e-01]
XSTD = [3.9612732767e+02, 1.8822821412e+04, 1.1226048640e+00, 6.8397462420e-01, 1.8879462146e+00,
        1.2433158499e+00, 1.3169176600e+00, 4.3600457243e-01, 8.1820904505e-01, 8.0471805333e-01,
        6.1020187522e-02]
YMU = [-0.0101101322, -0.0138129078, -0.0146349442, -0.0088870325, -0.0075195178, 0.0020506931, -0.0103104668,
       -0.0192603020]
YSTD = [0.0297933161, 0.0802139099, 0.0230954310, 0.1541940427, 0.1316836678, 0.0042975580, 0.1476416977,
        0.0860471308]
DIMS = [11, 1600, 800, 400, 1]


def _weights(seed=0):
    rng = np.random.default_rng(seed)
    mods = []
    for m in range(8):
        layers = []
        for l in range(4):
            fin, fout = DIMS[l], DIMS[l + 1]
            W = (rng.standard_normal((fout, fin)) / np.sqrt(fin)).astype(np.float32)
            b = (0.1 * rng.standard_normal(fout)).astype(np.float32)
            layers.append((W, b))
        mods.append(layers)
    return mods


def _torch_reference(mods, T, p, rho, Y, dt=1e-6, Tr=610.0):
    import torch
    S, C = Y.shape
    RR = np.zeros((S, C))
    react = T >= Tr
    Yr = Y[:, react]
    bct = (Yr ** 0.1 - 1) * 10
    x = np.concatenate([T[react][None, :], np.full((1, react.sum()), 101325.0), bct], axis=0).T
    x = (x - np.array(XMU)) / np.array(XSTD)
    xt = torch.tensor(x, dtype=torch.float32)
    yn = np.zeros((S - 1, react.sum()))
    for m, layers in enumerate(mods):
        h = xt
        for l, (W, b) in enumerate(layers):
            h = h @ torch.tensor(W).T + torch.tensor(b)
            if l < len(layers) - 1:
                h = torch.nn.functional.gelu(h)
        out = h[:, 0].double().numpy()
        yn[m] = ((out * YSTD[m] + YMU[m] + bct[m]) * 0.1 + 1) ** 10
    tot = yn.sum(axis=0) + Yr[S - 1]
    yn = yn / tot
    RR[:S - 1, react] = (yn - Yr[:S - 1]) * rho[react] * (p[react] / 101325.0) / dt
    return RR


def test_dnn_matches_torch_fp32():
    from dfmi.mesh import hex_box
    from dfmi.mech import read_thermo_table, read_yaml_mechanism
    from dfmi.lib import Context
    from dfmi import case
    ym = read_yaml_mechanism(os.path.join(GOLDEN, "Burke2012_s9r23.yaml"))
    t = read_thermo_table(os.path.join(GOLDEN, "thermo_Burke2012_s9r23.txt"), ym["species"])
    m = hex_box(16, 16, 8)
    ctx = Context(0)
    case.setup_context(ctx, m, t, ym["species"].index("N2"), 1e-6)
    mods = _weights()
    ctx.dnn_set_model(DIMS, mods, XMU, XSTD, YMU, YSTD)
    rng = np.random.default_rng(1)
    C = m.n_cells
    yu, yb = case.h2_air_compositions(ym["species"])
    prog = rng.random(C)
    Y = (1 - prog) * yu[:, None] + prog * yb[:, None] + 1e-4 * rng.random((9, C))
    Y /= Y.sum(axis=0)
    T = 300.0 + 2200.0 * rng.random(C)
    p = 101325.0 * (1 + 0.05 * rng.standard_normal(C))
    Wm = 1.0 / (Y / t.W[:, None]).sum(axis=0)
    rho = p * Wm / (8314.46261815324 * T)
    for n, v in (("T", T), ("p", p), ("rho", rho), ("Y", Y)):
        ctx.set_field(n, v)
    nr = ctx.dnn_infer()
    assert nr == int((T >= 610.0).sum())
    RR = ctx.get_field("RR", (9, C))
    ref = _torch_reference(mods, T, p, rho, Y)
    assert np.all(RR[:, T < 610.0] == 0.0)
    scale = np.abs(ref).max(axis=1, keepdims=True)[:8]
    err = np.abs(RR[:8] - ref[:8]) / scale
    assert np.all(np.isfinite(RR))
    assert np.median(err) < 2e-3, np.median(err)
    assert err.max() < 2e-2, err.max()
    _check_half_semantics(RR, mods, T, p, rho, Y, XMU, XSTD, YMU, YSTD)
    # heat release of the surrogate's source (pytorchFunctions.H:233-238) vs the oracle's sum over that RR
    from chem_oracle import heat_release, hf298_per_mass
    q = ctx.get_field("Qdot", (C,))
    qref = heat_release(hf298_per_mass(t.nasa, t.W), RR)
    assert np.array_equal(q, qref), np.abs(q - qref).max() / np.abs(qref).max()
    assert np.all(q[T < 610.0] == 0.0) and np.abs(q).max() > 0


def _half_reference(mods, T, p, rho, Y, xmu, xstd, ymu, ystd, dt=1e-6, Tr=610.0):
    """fp16-everywhere restatement on the GPU, as the reference runs it: modules_[i].to(device, kHalf)
    (dfChemistrySolver.cu:125), the normalised double input .to(kHalf) (:175), each net's output
    .to(kDouble) (:180) -- torch's own fp16 Linear (fp32 accumulation, fp16 output) and GELU"""
    import torch
    torch.backends.cuda.matmul.allow_fp16_reduced_precision_reduction = False
    S, C = Y.shape
    react = T >= Tr
    Yr = Y[:, react]
    bct = (Yr ** 0.1 - 1) * 10
    x = np.concatenate([T[react][None, :], np.full((1, react.sum()), 101325.0), bct], axis=0).T
    x = (x - np.asarray(xmu)) / np.asarray(xstd)
    xt = torch.tensor(x, dtype=torch.float64, device="cuda").to(torch.float16)
    yn = np.zeros((S - 1, react.sum()))
    with torch.no_grad():
        for m, layers in enumerate(mods):
            h = xt
            for l, (W, b) in enumerate(layers):
                Wt = torch.tensor(W, device="cuda").to(torch.float16)
                bt = torch.tensor(b, device="cuda").to(torch.float16)
                h = torch.nn.functional.linear(h, Wt, bt)
                if l < len(layers) - 1:
                    h = torch.nn.functional.gelu(h)
            out = h[:, 0].to(torch.float64).cpu().numpy()
            yn[m] = ((out * ystd[m] + ymu[m] + bct[m]) * 0.1 + 1) ** 10
    yn = yn / (yn.sum(axis=0) + Yr[S - 1])
    RR = np.zeros((S, C))
    RR[:S - 1, react] = (yn - Yr[:S - 1]) * rho[react] * (p[react] / 101325.0) / dt
    return RR


def _check_half_semantics(RR, mods, T, p, rho, Y, xmu, xstd, ymu, ystd):
    """per species, RR against the fp16-everywhere restatement: the kernel rounds where torch rounds
    (input, Linear output, GELU output, net output), so what remains is fp32 summation order and the
    erf approximation flipping the last fp16 bit of some activations"""
    S = Y.shape[0]
    ref = _half_reference(mods, T, p, rho, Y, xmu, xstd, ymu, ystd)
    scale = np.abs(ref).max(axis=1, keepdims=True)[:S - 1]
    err = np.abs(RR[:S - 1] - ref[:S - 1]) / scale
    per_species = err.max(axis=1)
    print("fp16-everywhere: median", np.median(err), "per-species max", per_species.max(),
          "exact fraction", float(np.mean(RR[:S - 1] == ref[:S - 1])))
    assert np.median(err) < 1e-4, np.median(err)
    assert per_species.max() < 4e-3, per_species


@pytest.mark.parametrize("tuned", [0, 1])
def test_dnn_53_species_matches_torch_fp32(tuned, monkeypatch):
    """BASELINE config 4's surrogate shape: 53 species, 52 nets [55, 1600, 800, 400, 1] with
    seeded weights and synthetic normalisation, on a small mesh; the context takes 53 species for the
    surrogate path (the FV kernels are not instantiated for it). tuned: the production shape-tuned kernels
    (option dnn.tuned_gemm = 1: the ping-pong 256x256x64 wide-layer kernel with tail strips, the 128x128
    input-layer kernel, the fused output layer) or k_mlp_gemm for every layer (0)."""
    import torch
    from dfmi import lib
    monkeypatch.setitem(lib.DEFAULT_OPTIONS, "dnn.tuned_gemm", tuned)
    from dfmi.mesh import hex_box
    from dfmi.lib import Context
    from dfmi import case, dnn_model
    S = 53
    m = hex_box(8, 8, 4)
    C = m.n_cells
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
    dims = [S + 2, 1600, 800, 400, 1]
    mods = dnn_model.seeded_weights(n_modules=S - 1, dims=dims, seed=2)
    xmu, xstd = np.zeros(S + 2), np.ones(S + 2)
    xmu[0], xstd[0], xmu[1], xstd[1] = 1300.0, 400.0, 101325.0, 1.0
    ymu, ystd = np.zeros(S - 1), np.full(S - 1, 0.01)
    ctx.dnn_set_model(dims, mods, xmu, xstd, ymu, ystd)
    rng = np.random.default_rng(4)
    Y = rng.gamma(0.3, 1.0, (S, C)) + 1e-8
    Y /= Y.sum(axis=0)
    T = 300.0 + 2200.0 * rng.random(C)
    p = 101325.0 * (1 + 0.05 * rng.standard_normal(C))
    rho = p / (300.0 * T)
    for n, v in (("T", T), ("p", p), ("rho", rho), ("Y", Y)):
        ctx.set_field(n, v)
    nr = ctx.dnn_infer()
    react = T >= 610.0
    assert nr == int(react.sum())
    RR = ctx.get_field("RR", (S, C))
    ctx.close()
    # torch fp32 restatement (dfChemistrySolver.cu:4-75 with these normalisation constants)
    Yr = Y[:, react]
    bct = (Yr ** 0.1 - 1) * 10
    x = np.concatenate([T[react][None, :], np.full((1, react.sum()), 101325.0), bct], axis=0).T
    xt = torch.tensor((x - xmu) / xstd, dtype=torch.float32)
    yn = np.zeros((S - 1, react.sum()))
    for k, layers in enumerate(mods):
        h = xt
        for l, (W, b) in enumerate(layers):
            h = h @ torch.tensor(W).T + torch.tensor(b)
            if l < len(layers) - 1:
                h = torch.nn.functional.gelu(h)
        out = h[:, 0].double().numpy()
        yn[k] = ((out * ystd[k] + ymu[k] + bct[k]) * 0.1 + 1) ** 10
    yn = yn / (yn.sum(axis=0) + Yr[S - 1])
    ref = np.zeros((S, C))
    ref[:S - 1, react] = (yn - Yr[:S - 1]) * rho[react] * (p[react] / 101325.0) / 1e-6
    assert np.all(RR[:, ~react] == 0.0) and np.all(np.isfinite(RR))
    scale = np.abs(ref).max(axis=1, keepdims=True)[:S - 1]
    err = np.abs(RR[:S - 1] - ref[:S - 1]) / scale
    assert np.median(err) < 2e-3, np.median(err)
    assert err.max() < 2e-2, err.max()
    _check_half_semantics(RR, mods, T, p, rho, Y, xmu, xstd, ymu, ystd)


def test_dnn_wide_layer_kernels_bitwise_at_scale(monkeypatch):
    """The 256x256x64 ping-pong wide-layer kernel (staggered wave groups, one-phase half-tile restaging, the
    800-wide layer's tail columns as two 16-column strips) and the 128x128 input-layer kernel (four workgroups per
    CU) issue the same MFMA sequence per output as k_mlp_gemm (option dnn.tuned_gemm = 0), so the source
    terms of 32,768 reacting cells x 52 nets agree bitwise -- a race in a pipeline's LDS reuse would show here
    (128 row tiles x 4 column tiles x 52 nets per launch, every CU busy)."""
    from dfmi.mesh import hex_box
    from dfmi.lib import Context
    from dfmi import case, dnn_model
    S = 53
    m = hex_box(32, 32, 32)
    C = m.n_cells
    dims = [S + 2, 1600, 800, 400, 1]
    mods = dnn_model.seeded_weights(n_modules=S - 1, dims=dims, seed=3)
    rng = np.random.default_rng(5)
    Y = rng.gamma(0.3, 1.0, (S, C)) + 1e-8
    Y /= Y.sum(axis=0)
    T = 800.0 + 1500.0 * rng.random(C)
    p = np.full(C, 101325.0)
    rho = p / (300.0 * T)
    out = {}
    from dfmi import lib
    for wide in ("0", "1"):
        monkeypatch.setitem(lib.DEFAULT_OPTIONS, "dnn.tuned_gemm", int(wide))
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
        xmu, xstd = np.zeros(S + 2), np.ones(S + 2)
        xmu[0], xstd[0], xmu[1], xstd[1] = 1300.0, 400.0, 101325.0, 1.0
        ctx.dnn_set_model(dims, mods, xmu, xstd, np.zeros(S - 1), np.full(S - 1, 0.01))
        for n, v in (("T", T), ("p", p), ("rho", rho), ("Y", Y)):
            ctx.set_field(n, v)
        assert ctx.dnn_infer() == C
        out[wide] = ctx.get_field("RR", (S, C))
        ctx.close()
    assert np.isfinite(out["0"]).all()
    assert np.array_equal(out["1"], out["0"]), np.abs(out["1"] - out["0"]).max()


def test_dnn_packed_model_file_equals_set_model(tmp_path):
    """dfmi_dnn_load_model (a packed file written from a reference-layout checkpoint, dfmi/dnn_checkpoint.py)
    installs exactly the model dfmi_dnn_set_model does: the same RR and Qdot bit for bit"""
    import torch
    from dfmi.mesh import hex_box
    from dfmi.mech import read_thermo_table, read_yaml_mechanism
    from dfmi.lib import Context
    from dfmi import case
    from dfmi.dnn_checkpoint import from_state_dict, write_packed
    ym = read_yaml_mechanism(os.path.join(GOLDEN, "Burke2012_s9r23.yaml"))
    t = read_thermo_table(os.path.join(GOLDEN, "thermo_Burke2012_s9r23.txt"), ym["species"])
    m = hex_box(16, 8, 8)
    C = m.n_cells
    mods = _weights()
    f64 = lambda v: torch.tensor(v, dtype=torch.float64)   # the normalisation stays double, as set_model takes it
    sd = {"data_in_mean": f64(XMU), "data_in_std": f64(XSTD), "data_target_mean": f64(YMU), "data_target_std": f64(YSTD)}
    for i, layers in enumerate(mods):
        sd[f"net{i}"] = {f"net.linear_layer_{k}.{n}": torch.from_numpy(a)
                         for k, (W, b) in enumerate(layers) for n, a in (("weight", W), ("bias", b))}
    path = tmp_path / "h2.dfmidnn"
    write_packed(str(path), from_state_dict(sd))
    rng = np.random.default_rng(4)
    yu, yb = case.h2_air_compositions(ym["species"])
    prog = rng.random(C)
    Y = (1 - prog) * yu[:, None] + prog * yb[:, None]
    Y /= Y.sum(axis=0)
    T = 300.0 + 2200.0 * rng.random(C)
    p = np.full(C, 101325.0)
    rho = p * (1.0 / (Y / t.W[:, None]).sum(axis=0)) / (8314.46261815324 * T)
    out = []
    for how in ("set", "file"):
        ctx = Context(0)
        case.setup_context(ctx, m, t, ym["species"].index("N2"), 1e-6)
        if how == "set":
            ctx.dnn_set_model(DIMS, mods, XMU, XSTD, YMU, YSTD)
        else:
            ctx.dnn_load_model(path)
        for n, v in (("T", T), ("p", p), ("rho", rho), ("Y", Y)):
            ctx.set_field(n, v)
        assert ctx.dnn_infer() == int((T >= 610.0).sum())
        out.append((ctx.get_field("RR", (9, C)), ctx.get_field("Qdot", (C,))))
        ctx.close()
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])
    assert np.abs(out[0][0]).max() > 0
