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


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64); b = np.asarray(b, dtype=np.float64)
    scale = max(np.abs(b).max(), 1e-300)
    return float(np.abs(a - b).max() / scale)
