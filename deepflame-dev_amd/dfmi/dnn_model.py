"""DF-ODENet surrogate configuration for the H2 (Burke 9-species) case.

The normalisation constants are the ones the reference hard-codes for its H2 nets
(src_gpu/dfChemistrySolver.cu:95-105); the layer widths are those of its NN_MLP
(test/Tu500K-Phi1/inference.py: [S+2, 1600, 800, 400, 1]). The trained weights are not in the
reference repository, so `seeded_weights` draws N(0, 1/fan_in) nets (seed fixed) --
same shapes and arithmetic, synthetic values."""
import numpy as np

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


def seeded_weights(n_modules=8, dims=DIMS, seed=0, out_scale=0.1):
    rng = np.random.default_rng(seed)
    mods = []
    for _ in range(n_modules):
        layers = []
        for l in range(len(dims) - 1):
            fin, fout = dims[l], dims[l + 1]
            W = (rng.standard_normal((fout, fin)) / np.sqrt(fin)).astype(np.float32)
            b = (0.1 * rng.standard_normal(fout)).astype(np.float32)
            if l == len(dims) - 2:
                W *= out_scale
            layers.append((W, b))
        mods.append(layers)
    return mods


def configure(ctx):
    ctx.dnn_set_model(DIMS, seeded_weights(), XMU, XSTD, YMU, YSTD)
