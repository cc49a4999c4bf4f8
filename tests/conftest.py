import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deepflame-dev_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
ROOT = ROOT
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libdfmi.so)")


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_first(request):
    """Some GPU tests compare against torch running on the device (the DNN's fp16 restatement). torch
    ships its own HIP runtime; it must initialise before libdfmi.so's, or torch finds no GPU (smoke() and
    bench.py initialise torch first as well)."""
    if any(item.get_closest_marker("gpu") for item in request.session.items):
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    yield


@pytest.fixture(scope="session")
def es80():
    from dfmi.mech import read_thermo_table, read_yaml_mechanism
    y = read_yaml_mechanism(os.path.join(GOLDEN, "ES80_H2-7-16.yaml"))
    t = read_thermo_table(os.path.join(GOLDEN, "thermo_ES80_H2-7-16.txt"), y["species"])
    return t, y


def ulp_diff(a, b):
    """max distance in units of the last place (0 = bit-identical)."""
    a = np.asarray(a, dtype=np.float64).ravel(); b = np.asarray(b, dtype=np.float64).ravel()
    ia = a.view(np.int64); ib = b.view(np.int64)
    ia = np.where(ia < 0, np.int64(-(2 ** 63)) - ia, ia)
    ib = np.where(ib < 0, np.int64(-(2 ** 63)) - ib, ib)
    return int(np.abs(ia - ib).max()) if a.size else 0


def rel_err(a, b, floor=1e-12):
    """max |a - b| relative to the reference's own magnitude, per component: a [k, n] field (vector
    components, species) is judged row by row against max |b_row|, so trace species (H2O2, HO2 at
    1e-6 of the major ones) are held to the same relative bar as the major ones. Rows whose magnitude
    is below `floor` x the field's maximum (identically-zero species) are judged against that floor."""
    a = np.asarray(a, dtype=np.float64); b = np.asarray(b, dtype=np.float64)
    if a.size == 0:
        return 0.0
    if b.ndim == 1:
        scale = max(np.abs(b).max(), 1e-300)
        return float(np.abs(a - b).max() / scale)
    a2 = a.reshape(a.shape[0], -1); b2 = b.reshape(b.shape[0], -1)
    top = max(np.abs(b2).max(), 1e-300)
    scale = np.maximum(np.abs(b2).max(axis=1), floor * top)
    return float((np.abs(a2 - b2).max(axis=1) / scale).max())
