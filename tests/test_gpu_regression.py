"""The reference's whole-loop regression on the GPU: test/dfLowMachFoam/twoD_reactingTGV/H2/cvodeSolver
(500 steps, its fvSchemes, ES80 chemistry at relTol 1e-9 / absTol 1e-15, cellPoint sampling) through
libdfmi.so, against the five values test/corrtest.cpp:52-56 asserts (0.5 %, see
tests/test_tgv2d_regression.py for the tolerance's basis) and against the committed CPU-A run of the same
case (tests/golden/tgv2d_cpu_a.json: the oracle's assembly; 1e-5 relative -- same discretisation, solvers
converged to 1e-10, device vs host libm in the chemistry)."""
import json
import os

import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def test_tgv2d_gpu_matches_reference_regression():
    from dfmi import regression as R
    out = R.run_tgv2d(os.path.join(GOLDEN, "tgv2d"), GOLDEN, log=print)
    ref = json.load(open(os.path.join(GOLDEN, "tgv2d_cpu_a.json")))["steps"]
    for step, r in out.items():
        dev = abs(r["value"] - r["expected"]) / r["expected"]
        assert dev < 5e-3, (step, r["value"], r["expected"], dev)
        cpu = ref[str(step)]["value"]
        assert abs(r["value"] - cpu) < 1e-5 * cpu, (step, r["value"], cpu)


def test_flame_speed_gpu_matches_reference_regression():
    """test/Tu500K-Phi1 for 2 ms (2000 steps) on the GPU: the flameSpeed utility's value for 1 -> 2 ms
    against corrtest.cpp:269-270's 6 m/s within 0.2 m/s (see tests/test_flame_speed_regression.py), and the
    flame positions equal to CPU-A's (the same cells)."""
    from dfmi import regression as R
    out = R.run_flame1d_speed(GOLDEN, log=print)
    fs = out["flameSpeed"][2000]
    assert abs(fs - R.FLAME_SPEED_EXPECTED) <= 0.2, out
    ref = json.load(open(os.path.join(GOLDEN, "flame1d_speed_cpu_a.json")))
    for k, x in out["positions"].items():
        assert abs(x - ref["positions"][str(k)]) < 1e-9, (k, x, ref["positions"])
