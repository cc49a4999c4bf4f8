"""The reference's flame-speed regression on the CPU (CPU-A): test/Tu500K-Phi1 (880 cells, Burke2012 9
species, its 0/ fields, fvSchemes incl. div(phi,U) limitedLinearV 1, waveTransmissive outlet) run for 2 ms,
the flame position (cell of max dT/dx) read as applications/utilities/flameSpeed/flameSpeed.C:48-72 does,
against corrtest.cpp:269-270 (fs = 6 m/s for the 1 -> 2 ms interval).

Tolerance 0.2 m/s. The measurement's quantum is one cell per millisecond (40 um / 1 ms = 0.04 m/s in
the uniform section). The reference number was produced with the DF-ODENet surrogate (the CI builds with
--use_pytorch and the case sets TorchSettings torch on; pytorchFunctions.H solve_DNN), whose trained weights
are not in the repository; we integrate the chemistry the surrogate replaces (ROS3, odeCoeffs 1e-6 /
1e-10). Measured: 6.00 m/s for 0 -> 1 ms, 5.84 m/s for 1 -> 2 ms (4 cells from the reference's 16-cell
move), independent of the schemes (upwind/linear moves the flame through the same cells).

This is a loose pin, not parity: the reference asserts EXPECT_FLOAT_EQ(fs, 6) on its DNN-driven run, and
flame-speed parity with the reference stays unpinned without the surrogate's weights. What is pinned exactly
is our own consistency: the GPU run's flame positions equal CPU-A's cell for cell
(tests/test_gpu_regression.py), as this file's CPU rerun checks against the committed CPU-A positions.
"""
import json
import os

import pytest

from conftest import GOLDEN, ROOT

CPU_A = os.path.join(ROOT, "baseline", "cpu_a", "libdfmi_cpu_a.so")


def test_committed_cpu_a_flame_speed():
    """the committed CPU-A run (tests/golden/flame1d_speed_cpu_a.json) meets corrtest.cpp:269-270"""
    from dfmi import regression as R
    ref = json.load(open(os.path.join(GOLDEN, "flame1d_speed_cpu_a.json")))
    assert abs(ref["flameSpeed"]["2000"] - R.FLAME_SPEED_EXPECTED) <= 0.2, ref


@pytest.mark.skipif(os.environ.get("DFMI_REGRESSION") != "1",
                    reason="2000-step CPU-A rerun (minutes): set DFMI_REGRESSION=1; the GPU test reruns it")
def test_flame_speed_cpu_matches_reference_regression():
    from dfmi import regression as R
    if not os.path.exists(CPU_A):
        pytest.skip("CPU-A not built")
    out = R.run_flame1d_speed(GOLDEN, lib_path=CPU_A)
    fs = out["flameSpeed"][2000]
    assert abs(fs - R.FLAME_SPEED_EXPECTED) <= 0.2, out
    ref = json.load(open(os.path.join(GOLDEN, "flame1d_speed_cpu_a.json")))
    for k, x in out["positions"].items():
        assert abs(x - ref["positions"][str(k)]) < 1e-9, (k, x)
