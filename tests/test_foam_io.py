"""OpenFOAM ASCII field I/O on the reference example's own 0/ fields
(examples/dfLowMachFoam/notorch/threeD_reactingTGV/H2/cvodeIntegrator/0, committed under
tests/golden/tgv64), and the 2x2x2 tiling of BASELINE config 3."""
import os

import numpy as np

from conftest import GOLDEN


def test_read_reference_tgv_fields():
    from dfmi.foam_io import read_case_fields, read_field
    from dfmi.mech import read_yaml_mechanism
    ym = read_yaml_mechanism(os.path.join(GOLDEN, "Burke2012_s9r23.yaml"))
    f = read_case_fields(os.path.join(GOLDEN, "tgv64"), ym["species"])
    assert f["T"].shape == (64 ** 3,) and f["U"].shape == (3, 64 ** 3) and f["Y"].shape == (9, 64 ** 3)
    assert 300.0 <= f["T"].min() < 300.001 and 1848.0 < f["T"].max() < 1849.0
    assert np.allclose(f["Y"].sum(axis=0), 1.0, atol=1e-12)
    assert np.all(f["p"] == 101325.0)
    _, types = read_field(os.path.join(GOLDEN, "tgv64", "T.gz"))
    assert set(types.values()) == {"cyclic"} and len(types) == 6


def test_tiling_and_roundtrip(tmp_path):
    from dfmi.foam_io import tile_fields, write_field, read_field
    rng = np.random.default_rng(0)
    f = {"T": rng.random(4 ** 3), "U": rng.random((3, 4 ** 3))}
    g = tile_fields(f, 4)
    T = g["T"].reshape(8, 8, 8)
    assert np.array_equal(T[:4, :4, :4], T[4:, 4:, 4:]) and np.array_equal(T[:4, :4, :4].ravel(), f["T"])
    assert np.array_equal(g["U"][:, :4], f["U"][:, :4])
    p = str(tmp_path / "T.gz")
    write_field(p, "T", f["T"], {"left": "cyclic"})
    v, t = read_field(p)
    assert np.array_equal(v, f["T"]) and t == {"left": "cyclic"}
    p = str(tmp_path / "U")
    write_field(p, "U", f["U"].T, {"w": "zeroGradient"})
    v, _ = read_field(p)
    assert np.array_equal(v, f["U"].T)


def test_flame1d_case_fixture():
    """BASELINE config 2 inputs: the reference 1D flame's 0/ files (tests/golden/flame1d) and its
    blockMesh multi-grading ((0.55 0.625 1) (0.45 0.375 2)) over 40 mm / 880 cells."""
    import numpy as np
    from dfmi import case
    from dfmi.foam_io import read_boundary
    from dfmi.mech import read_yaml_mechanism
    ym = read_yaml_mechanism(os.path.join(GOLDEN, "Burke2012_s9r23.yaml"))
    m = case.flame1d_mesh()
    x = np.concatenate([[0.0], np.cumsum(m.volume / 1e-6)])          # cell widths (1 mm x 1 mm section)
    d = np.diff(x)
    assert m.n_cells == 880 and m.n_faces == 879 and m.n_boundary_slots == 2
    assert abs(x[550] - 0.022) < 1e-12 and abs(x[-1] - 0.04) < 1e-12   # 55 % of the length in 62.5 % of the cells
    assert np.allclose(d[:550], 0.022 / 550) and abs(d[-1] / d[550] - 2.0) < 1e-9
    f, bv = case.flame1d_fields(os.path.join(GOLDEN, "flame1d"), ym["species"])
    assert f["T"].shape == (880,) and f["T"].min() == 500.0 and abs(f["T"].max() - 2485.8) < 1e-9
    assert np.allclose(f["Y"].sum(axis=0), 1.0, atol=1e-12)
    assert bv["T"]["left"] == 500.0 and bv["p"]["right"] == 101325.0
    assert np.allclose(bv["U"]["left"], [5.36, 0, 0]) and abs(bv["Y"]["left"].sum() - 1.0) < 1e-12
    b = read_boundary(os.path.join(GOLDEN, "flame1d", "p"))
    assert b["outlet"] == ("waveTransmissive", 101325.0) and b["boundary"][0] == "empty"
