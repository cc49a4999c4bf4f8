"""DF-ODENet weight ingestion (VERDICT r05 missing 3): a checkpoint in the reference's layout
(test/Tu500K-Phi1/inference.py:12-25,76-106 -- one dict with the normalisation vectors and a NN_MLP state_dict
per species under net<i>) read weights-only and packed into exactly the arrays dfmi_dnn_set_model takes. The
reference's trained weights are absent, so the checkpoint here is synthetic: the seeded nets of
dfmi/dnn_model.py loaded into real torch NN_MLP modules and saved with torch.save."""
import os

import numpy as np
import pytest



def _nn_mlp(layer_info):
    """inference.py's NN_MLP: a Sequential attribute `net` of linear_layer_<k> / gelu_layer_<k>"""
    import torch

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.net = torch.nn.Sequential()
            n = len(layer_info) - 1
            for i in range(n - 1):
                self.net.add_module("linear_layer_%d" % i, torch.nn.Linear(layer_info[i], layer_info[i + 1]))
                self.net.add_module("gelu_layer_%d" % i, torch.nn.GELU())
            self.net.add_module("linear_layer_%d" % (n - 1), torch.nn.Linear(layer_info[n - 1], layer_info[n]))
    return M()


def _checkpoint(mods, dims, xmu, xstd, ymu, ystd):
    import torch
    sd = {"data_in_mean": np.asarray(xmu), "data_in_std": np.asarray(xstd),
          "data_target_mean": np.asarray(ymu), "data_target_std": np.asarray(ystd)}
    for i, layers in enumerate(mods):
        net = _nn_mlp(dims)
        with torch.no_grad():
            for k, (W, b) in enumerate(layers):
                lin = getattr(net.net, "linear_layer_%d" % k)
                lin.weight.copy_(torch.from_numpy(W))
                lin.bias.copy_(torch.from_numpy(b))
        sd[f"net{i}"] = net.state_dict()
    return sd


@pytest.fixture(scope="module")
def small():
    from dfmi.dnn_model import XMU, XSTD, YMU, YSTD, seeded_weights
    dims = [11, 32, 16, 8, 1]   # the H2 input width with narrow hidden layers (the layout, not the size, is tested)
    return dims, seeded_weights(8, dims, seed=5), XMU, XSTD, YMU, YSTD


def test_checkpoint_round_trip_packs_the_set_model_arrays(small, tmp_path):
    import torch
    from dfmi.dnn_checkpoint import pack_params, read_checkpoint, read_packed, write_packed
    dims, mods, xmu, xstd, ymu, ystd = small
    path = tmp_path / "DNN_model.pt"
    torch.save(_checkpoint(mods, dims, xmu, xstd, ymu, ystd), path)
    m = read_checkpoint(str(path))
    assert m["dims"] == dims and len(m["params"]) == 8
    # the packed parameters are the array dfmi.lib.Context.dnn_set_model hands the library for the same nets
    assert np.array_equal(pack_params(m["params"]), pack_params(mods))
    for k, v in (("x_mu", xmu), ("x_std", xstd), ("y_mu", ymu), ("y_std", ystd)):
        assert np.array_equal(m[k], np.asarray(v, dtype=np.float64))
    out = tmp_path / "model.dfmidnn"
    write_packed(str(out), m)
    r = read_packed(str(out))
    assert r["dims"] == dims and r["n_modules"] == 8
    assert np.array_equal(r["flat"], pack_params(mods))
    assert np.array_equal(r["x_std"], np.asarray(xstd)) and np.array_equal(r["y_mu"], np.asarray(ymu))


def test_full_width_h2_layout(tmp_path):
    """the reference's own widths [S + 2, 1600, 800, 400, 1] for the 9-species H2 case"""
    import torch
    from dfmi.dnn_checkpoint import pack_params, read_checkpoint
    from dfmi.dnn_model import DIMS, XMU, XSTD, YMU, YSTD, seeded_weights
    mods = seeded_weights()
    path = tmp_path / "h2.pt"
    torch.save(_checkpoint(mods, DIMS, XMU, XSTD, YMU, YSTD), path)
    m = read_checkpoint(str(path))
    assert m["dims"] == DIMS
    assert np.array_equal(pack_params(m["params"]), pack_params(mods))


def test_checkpoint_that_executes_code_is_refused(tmp_path):
    """weights_only loading: a pickled object (anything beyond tensors / containers) is not unpickled"""
    import torch
    from dfmi.dnn_checkpoint import read_checkpoint

    class Payload:
        def __reduce__(self):
            return (os.getcwd, ())
    path = tmp_path / "evil.pt"
    torch.save({"data_in_mean": Payload()}, path)
    with pytest.raises(ValueError, match="weights-only"):
        read_checkpoint(str(path))


def test_layout_errors_are_reported(small, tmp_path):
    from dfmi.dnn_checkpoint import from_state_dict
    dims, mods, xmu, xstd, ymu, ystd = small
    sd = _checkpoint(mods, dims, xmu, xstd, ymu, ystd)
    bad = dict(sd)
    del bad["net3"]
    with pytest.raises(ValueError, match="net0 .. net"):
        from_state_dict(bad)
    bad = dict(sd)
    bad["data_target_mean"] = np.zeros(7)
    with pytest.raises(ValueError, match="data_target_mean"):
        from_state_dict(bad)
    bad = dict(sd)
    bad.pop("data_in_std")
    with pytest.raises(ValueError, match="lacks"):
        from_state_dict(bad)
    bad = dict(sd)
    net = dict(bad["net1"])
    net["net.linear_layer_9.weight"] = net.pop("net.linear_layer_3.weight")
    bad["net1"] = net
    with pytest.raises(ValueError):
        from_state_dict(bad)
