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
